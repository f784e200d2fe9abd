#!/usr/bin/env python3
"""Build F-Stack's kernel domain with IPsec and the MI355X driver into an
executable that runs the reference's own opencrypto framework
(integration/fstack_run/, INTEGRATION.md section 4, "Running it").

    python integration/fstack_run.py build [--ref /root/reference] [--work DIR]

1. integration/fstack_build_check.py's build_kernel(): the F-Stack tree
   copied and patched (apply_fstack.sh), every kernel-domain object of an
   `FF_IPSEC=1 FF_IPSEC_GPU=1` build compiled by lib/Makefile's own rules,
   plus fstack_run/ff_crypto_selftest.c with the same NORMAL_C command;
2. libfstack.a's recipe (lib/Makefile:673-680): `ld -d -r` of those objects,
   every symbol localised, then ff_api.symlist (plus the selftest's ffst_*
   entry points) made global again;
3. the host domain: fstack_run/host_main.c and fstack_run/host_stubs.c (the
   DPDK-side symbols, integration/fstack_build_check.py "host_blocked"),
   with either the real host shim ff_gpucrypto_host.c + libespgpu.so
   (integration/fstack_crypto_run_gpu) or the oracle stand-in
   fstack_run/oracle_engine.c (integration/fstack_crypto_run_cpu).
The executables are built here (they need /root/reference) and, like the
.so files, travel to the GPU box untracked.

pack_requests() / read_results() are the file formats host_main.c reads and
writes (used by tests/test_fstack_run.py).
"""
import argparse
import os
import struct
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
RUN = os.path.join(HERE, "fstack_run")
EXE_CPU = os.path.join(HERE, "fstack_crypto_run_cpu")
EXE_GPU = os.path.join(HERE, "fstack_crypto_run_gpu")
EXPORTS = ["ffst_find_driver", "ffst_newsession", "ffst_freesession", "ffst_request", "ffst_dispatch",
           "ffst_result", "ffst_ndone", "ffst_redispatch", "ffst_free"]
SELFTEST_RULE = """
ff_crypto_selftest.o: ff_crypto_selftest.c $(IMACROS_FILE)
\t${NORMAL_C}
"""


def run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{' '.join(cmd)}: rc {r.returncode}\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}")
    return r


def build(ref, work, jobs=8):
    sys.path.insert(0, HERE)
    import fstack_build_check as B
    lib, make, objs, report, rc = B.build_kernel(ref, work, jobs, extra_make=SELFTEST_RULE)
    if rc != 0:
        raise RuntimeError("kernel-domain compile failed: %s" % report["compile_errors"][:5])
    import shutil
    shutil.copy(os.path.join(RUN, "ff_crypto_selftest.c"), lib)
    run(make + ["ff_crypto_selftest.o"], cwd=lib)
    # libfstack.a's recipe: incremental link, localise everything, globalise the API
    ro = os.path.join(work, "libfstack_run.ro")
    run(["ld", "-d", "-r", "-o", ro] + objs + ["ff_crypto_selftest.o"], cwd=lib)
    defined = [l.split()[-1] for l in run(["nm", ro]).stdout.splitlines() if len(l.split()) == 3]
    loc = os.path.join(work, "localize.txt")
    open(loc, "w").write("\n".join(defined) + "\n")
    run(["objcopy", "--localize-symbols=" + loc, ro])
    glob = os.path.join(work, "globalize.txt")
    api = open(os.path.join(lib, "ff_api.symlist")).read().split()
    open(glob, "w").write("\n".join(api + EXPORTS) + "\n")
    run(["objcopy", "--globalize-symbols=" + glob, ro])
    # host domain, with lib/Makefile's HOST_CFLAGS
    host_c = run(make + ["print-host-c"], cwd=lib).stdout.split()
    inc = ["-I" + lib, "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "oracle")]
    objs_h = {}
    for name, src, defs in (("stubs", os.path.join(RUN, "host_stubs.c"), []),
                            ("main_cpu", os.path.join(RUN, "host_main.c"), []),
                            ("main_gpu", os.path.join(RUN, "host_main.c"), ["-DFSR_GPU"]),
                            ("oracle_engine", os.path.join(RUN, "oracle_engine.c"), []),
                            ("shim", os.path.join(HERE, "ff_gpucrypto_host.c"), [])):
        o = os.path.join(work, name + ".host.o")
        run(host_c + defs + inc + [src, "-o", o], cwd=lib)
        objs_h[name] = o
    espgpu = os.path.join(ROOT, "f-stack_amd")
    orc = os.path.join(ROOT, "oracle")
    common = ["-no-pie", ro, objs_h["stubs"], "-L" + espgpu, "-lespgpu", "-Wl,-rpath," + espgpu, "-lpthread", "-lm"]
    run(["gcc", "-o", EXE_CPU, objs_h["main_cpu"], objs_h["oracle_engine"]] + common +
        ["-L" + orc, "-loracle", "-Wl,-rpath," + orc])
    run(["gcc", "-o", EXE_GPU, objs_h["main_gpu"], objs_h["shim"]] + common)
    return EXE_CPU, EXE_GPU


# ---------------------------------------------------------------------------
# file formats (host_main.c)

def pack_requests(path, sessions, requests):
    """sessions: dicts mode, flags, ivlen, calg, cklen, aalg, aklen, mlen,
    ckey, akey.  requests: dicts ses, op, flags, aad_start, aad_len,
    iv_start, payload_start, payload_len, digest_start, aad (bytes | None),
    esn (4 bytes), iv (bytes | None), mbuf (bool), cuts (list), buf (bytes)."""
    with open(path, "wb") as f:
        f.write(struct.pack("<III", 0x52435346, len(sessions), len(requests)))
        for s in sessions:
            f.write(struct.pack("<8i", s["mode"], s["flags"], s["ivlen"], s["calg"], s["cklen"], s["aalg"],
                                s["aklen"], s["mlen"]))
            f.write(bytes(s.get("ckey") or b"").ljust(32, b"\0")[:32])
            f.write(bytes(s.get("akey") or b"").ljust(128, b"\0")[:128])
        for r in requests:
            cuts = list(r.get("cuts") or [])
            assert len(cuts) <= 16
            aad = r.get("aad")
            iv = r.get("iv")
            f.write(struct.pack("<12i", r["ses"], r["op"], r["flags"], r["aad_start"], r["aad_len"], r["iv_start"],
                                r["payload_start"], r["payload_len"], r["digest_start"], int(aad is not None),
                                int(iv is not None), int(bool(r.get("mbuf")))))
            f.write(bytes(aad or b"").ljust(16, b"\0")[:16])
            f.write(bytes(r.get("esn") or b"\0\0\0\0")[:4].ljust(4, b"\0"))
            f.write(bytes(iv or b"").ljust(16, b"\0")[:16])
            f.write(struct.pack("<i16i", len(cuts), *(cuts + [0] * (16 - len(cuts)))))
            f.write(struct.pack("<i", len(r["buf"])))
            f.write(bytes(r["buf"]))


def read_results(path, lens, fail=False):
    """-> (gpu_hid, sw_hid, sessions [(err_def, hid_def, err_sw, hid_sw)],
    requests [dict etype, done_flag, buf, etype_sw, done_flag_sw, buf_sw,
    dispatch, dispatch_sw]; with fail (host_main.c --fail) also f1_dispatch,
    f1_ndone0, f1_etype0, f1_ndone, f1_etype, f1_buf (dispatched as the GPU
    failed: held, or refused and moved), f2_redispatch, f2_etype0, f2_hid,
    f2_ndone, f2_etype, f2_buf (dispatched after it)]"""
    with open(path, "rb") as f:
        magic, nses, nreq, gh, sh = struct.unpack("<IIIii", f.read(20))
        assert magic == 0x53525346 and nreq == len(lens)
        ses = [struct.unpack("<4i", f.read(16)) for _ in range(nses)]
        reqs = []
        for n in lens:
            v = struct.unpack("<6i", f.read(24))
            b0, b1 = f.read(n), f.read(n)
            d = dict(etype=v[0], done_flag=v[1], buf=b0, etype_sw=v[2], done_flag_sw=v[3], buf_sw=b1,
                     dispatch=v[4], dispatch_sw=v[5])
            if fail:
                w = struct.unpack("<10i", f.read(40))
                d.update(f1_dispatch=w[0], f1_ndone0=w[1], f1_etype0=w[2], f1_ndone=w[3], f1_etype=w[4],
                         f2_redispatch=w[5], f2_etype0=w[6], f2_hid=w[7], f2_ndone=w[8], f2_etype=w[9],
                         f1_buf=f.read(n), f2_buf=f.read(n))
            reqs.append(d)
    return gh, sh, ses, reqs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build"])
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--work", default="/tmp/fstack_run_build")
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args()
    print(build(a.ref, a.work, a.j))


if __name__ == "__main__":
    main()
