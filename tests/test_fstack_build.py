"""F-Stack's FF_IPSEC=1 FF_IPSEC_GPU=1 build, kernel domain, compiled and
link-checked here (integration/fstack_build_check.py).

The reference's FF_IPSEC build is broken: an empty
CRYPTO_SRCS, sources that are not in the tree (blowfish) or need compiler
intrinsics under -nostdinc (aesni_wrap.c), gmac.c/gfmult.c, subr_ipsec.c and
ipsec_mod.c missing, no kproc_create, no newbus to run crypto_init.  With
integration/fstack-ipsec-gpu.patch every kernel-domain object of that build
(lib/Makefile's own NORMAL_C rule: -nostdinc, FreeBSD headers, -Werror)
compiles, including the non-KMOCK ff_gpucrypto.c and ff_newbus.c, and every
symbol still undefined after `ld -r` is linker-generated, libc's, or defined by
an F-Stack host-domain source."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "lib")), reason="needs the F-Stack tree")
def test_fstack_ipsec_gpu_kernel_domain_compiles_and_links(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "integration", "fstack_build_check.py"),
                        "--ref", REF, "--work", str(tmp_path / "fs"), "-j", "8"],
                       capture_output=True, text=True, timeout=600)
    assert r.stdout.strip(), r.stderr[-3000:]
    rep = json.loads(r.stdout)
    assert rep["compile_errors"] == [], rep["compile_errors"][:20]
    assert rep["unresolved"] == [], rep["unresolved"]
    assert rep["missing_exports"] == []
    assert r.returncode == 0
    assert rep["kernel_objects"] > 200
    # the driver's calls into the host domain resolve to the host shim
    assert set(rep["gpu_driver_calls_host"]) == {
        "ff_gpucrypto_host_probe", "ff_gpucrypto_host_newsession", "ff_gpucrypto_host_freesession",
        "ff_gpucrypto_host_process", "ff_gpucrypto_host_ready", "ff_gpucrypto_host_failed"}
    assert "ff_gpucrypto_host.c" in rep["host_compiled"]
    # host files that need DPDK headers are named with the header that blocks them
    assert rep["host_blocked"].get("ff_dpdk_if.c", "").startswith("rte_")
