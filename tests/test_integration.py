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


def test_kernel_driver_errno_and_erestart():
    _make()
    r = subprocess.run([os.path.join(D, "kmock_cpu_test")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "kmock cpu OK" in r.stdout


@pytest.mark.gpu
def test_kernel_driver_on_gpu():
    exe = os.path.join(D, "kmock_gpu_test")
    assert os.path.exists(exe), "build() / make -C integration first"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "kmock gpu OK" in r.stdout
