"""The F-Stack host-domain binding (integration/ff_gpucrypto_host.c, the C a
maintainer adds as an FF_HOST_SRCS file per INTEGRATION.md) compiles against
include/espgpu.h, links against libespgpu.so, and its device-free entry
points (ABI version, CRYPTODEV_PROBESESSION, poll without a context) behave."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_shim_builds_links_and_probes():
    d = os.path.join(ROOT, "integration")
    subprocess.run(["make", "-s", "-C", d], check=True, timeout=300)
    r = subprocess.run([os.path.join(d, "probe_check")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "integration probe OK" in r.stdout
