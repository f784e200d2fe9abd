"""The F-Stack binding, built outside F-Stack:

* integration/ff_gpucrypto_host.c (host domain) compiles against
  include/espgpu.h, links against libespgpu.so, and its device-free entry
  points behave (probe_check);
* integration/ff_gpucrypto.c, the kernel-domain opencrypto driver, over the
  kmock crypto KPI and a scripted host layer: CRYPTOCAP_F_HARDWARE|SYNC at
  attach, the ABI -> FreeBSD errno map, ERESTART reaching the framework as
  ERESTART (-1) with the request queued and retried after crypto_unblock,
  an ICV failure completing with crp_etype 89 (kmock_cpu_test);
* the same driver over the real host shim and engine on the GPU, with a
  staging area small enough that a burst is ERESTARTed (kmock_gpu_test)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
D = os.path.join(ROOT, "integration")


def _make():
    subprocess.run(["make", "-s", "-C", D], check=True, timeout=300)


def test_host_shim_builds_links_and_probes():
    _make()
    r = subprocess.run([os.path.join(D, "probe_check")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "integration probe OK" in r.stdout


def test_kernel_driver_errno_erestart_and_gpu_failure():
    """kmock_cpu_test: the driver over the kmock KPI and the scripted host
    layer -- attach flags, errno map, ERESTART queueing, and the GPU-failure
    path: staged requests complete exactly once with EIO, the next request
    of a session moves it to the software driver (EAGAIN + new session),
    new sessions go there, every session is freed."""
    _make()
    r = subprocess.run([os.path.join(D, "kmock_cpu_test")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "kmock cpu OK" in r.stdout


def test_kernel_driver_python_harness_builds():
    """integration/libkmockdrv.so (ff_gpucrypto.c over kmock + the host shim,
    flat entry points for tests/test_kmock_driver_gpu.py) builds, loads and
    exports them (no compute calls: no GPU here)."""
    import ctypes
    _make()
    L = ctypes.CDLL(os.path.join(D, "libkmockdrv.so"))
    for s in ("kd_open", "kd_close", "kd_newsession", "kd_freesession", "kd_request", "kd_dispatch",
              "kd_poll", "kd_result", "kd_free", "kd_register", "kd_counters", "kd_engine",
              "kd_tune", "kd_failed", "kd_done_count", "kd_session_hid", "kd_redispatch", "kd_soft_enable",
              "kd_soft", "kd_freesession_of"):
        assert hasattr(L, s), s


@pytest.mark.gpu
def test_kernel_driver_on_gpu():
    exe = os.path.join(D, "kmock_gpu_test")
    assert os.path.exists(exe), "build() / make -C integration first"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "kmock gpu OK" in r.stdout


REF_LIB = "/root/reference/lib"


def _makefile_block(text, start, stop="endif"):
    """The reference Makefile's `start ... stop` block, verbatim."""
    i = text.index(start)
    return text[i:text.index("\n" + stop, i) + len(stop) + 1] + "\n"


@pytest.mark.skipif(not os.path.isdir(REF_LIB), reason="needs the F-Stack tree")
def test_fstack_patch_applies_and_fixes_the_ipsec_build(tmp_path):
    """integration/apply_fstack.sh on a copy of the F-Stack files it touches:
    the patch applies cleanly, the driver and shim land in lib/, and GNU make
    evaluates the patched FF_IPSEC blocks to the sources the path needs (the
    unpatched `#aesni.c \\` line empties CRYPTO_SRCS; xform.c
    needs gmac.c/gfmult.c; FF_IPSEC_GPU adds the driver, shim and include)."""
    import shutil
    lib = tmp_path / "lib"
    lib.mkdir()
    for f in ("Makefile", "ff_api.symlist", "ff_dpdk_if.c", "ff_init.c", "ff_compat.c", "ff_glue.c",
              "ff_host_interface.c", "ff_host_interface.h"):
        shutil.copy(os.path.join(REF_LIB, f), lib / f)
    sh = os.path.join(D, "apply_fstack.sh")
    subprocess.run(["sh", sh, str(tmp_path), "--dry-run"], check=True, capture_output=True, timeout=60)
    subprocess.run(["sh", sh, str(tmp_path)], check=True, capture_output=True, timeout=60)
    assert (lib / "ff_gpucrypto.c").exists() and (lib / "ff_gpucrypto_host.c").exists()

    def evaluate(mk_text, defs):
        frag = tmp_path / "frag.mk"
        frag.write_text(mk_text + "\nprint:\n\t@echo CRYPTO=$(strip $(CRYPTO_SRCS))"
                        "\n\t@echo OPENCRYPTO=$(strip $(OPENCRYPTO_SRCS))"
                        "\n\t@echo FF=$(strip $(FF_SRCS))\n\t@echo HOST=$(strip $(FF_HOST_SRCS))"
                        "\n\t@echo CFLAGS=$(strip $(CFLAGS))\n")
        r = subprocess.run(["make", "-s", "-f", str(frag), "print"] + defs, capture_output=True,
                           text=True, timeout=60, check=True)
        return dict(l.split("=", 1) for l in r.stdout.splitlines())

    orig = open(os.path.join(REF_LIB, "Makefile")).read()
    new = (lib / "Makefile").read_text()
    before = evaluate(_makefile_block(orig, "ifdef FF_IPSEC\nCRYPTO_SRCS"), ["FF_IPSEC=1"])
    assert before["CRYPTO"] == ""                         # the reference bug, reproduced
    blocks = (_makefile_block(new, "ifdef FF_IPSEC\nCRYPTO_SRCS") +
              _makefile_block(new, "ifdef FF_IPSEC\nOPENCRYPTO_SRCS") +
              new[new.index("ifdef FF_IPSEC_GPU"):new.index("#\tcryptodev.c")])
    after = evaluate(blocks, ["FF_IPSEC=1", "FF_IPSEC_GPU=1", "ESPGPU_ROOT=/opt/espgpu"])
    assert {"rijndael-alg-fst.c", "rijndael-api.c", "sha1.c", "sha256c.c", "sha512c.c"} <= set(after["CRYPTO"].split())
    assert {"gmac.c", "gfmult.c", "cryptosoft.c", "crypto.c"} <= set(after["OPENCRYPTO"].split())
    assert after["FF"].split() == ["ff_gpucrypto.c"] and after["HOST"].split() == ["ff_gpucrypto_host.c"]
    assert "-I/opt/espgpu/include" in after["CFLAGS"] and "-DFF_IPSEC_GPU" in after["CFLAGS"]

    syms = (lib / "ff_api.symlist").read_text().split()
    assert {"ff_gpucrypto_done", "ff_gpucrypto_unblock"} <= set(syms)
    loop = (lib / "ff_dpdk_if.c").read_text()
    i = loop.index("process_msg_ring(qconf->proc_id, pkts_burst);")
    assert loop.index("ff_gpucrypto_poll();", i) < loop.index("lr->loop(lr->arg)", i)
    init = (lib / "ff_init.c").read_text()
    # the GPU context exists before ff_freebsd_init() attaches the drivers
    assert (init.index("ret = ff_dpdk_init(") < init.index("ff_gpucrypto_host_init_proc(ff_global_cfg")
            < init.index("ret = ff_freebsd_init();"))
    # the mbuf pools (made by ff_dpdk_init) are mapped for the GPU once the context exists
    assert (init.index("ff_gpucrypto_host_init_proc(ff_global_cfg") < init.index("ff_dpdk_register_gpu_mem()")
            < init.index("ret = ff_freebsd_init();"))
    assert "rte_mempool_mem_iter(pktmbuf_pool[i], ff_gpucrypto_mem_cb" in loop
    assert (lib / "ff_newbus.c").exists()
