"""pytest setup: import paths, the `gpu` marker, and on-demand native builds.

The native artefacts (.so) are git-ignored; they are rebuilt here if missing
so a fresh checkout runs.  `make` is incremental, so this is a no-op when the
libraries are up to date.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "f-stack_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def _make(args, fatal=True):
    try:
        subprocess.run(["make", "-s"] + args, cwd=ROOT, check=True, timeout=900,
                       stdout=subprocess.DEVNULL)
    except Exception as e:
        msg = "conftest: make %s failed: %s" % (" ".join(args), e)
        if fatal:   # never test a stale library
            raise RuntimeError(msg)
        print(msg, file=sys.stderr)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    _make(["-C", "oracle", "liboracle.so"])
    if os.path.isdir("/root/reference/freebsd"):
        _make(["-C", "oracle", "ref"], fatal=False)
    _make(["-C", "f-stack_amd", "-j8"])


@pytest.fixture(params=[4, 8], ids=["lanes4", "lanes8"])
def gcm_lanes(request, drv):
    """Run a GCM test through both kernels whatever its batch size: 4 lanes
    per record (the throughput kernel) and 8 (the small-batch kernel, half
    the serial steps); set_tuning "gcm_lanes", reset afterwards."""
    assert drv.lib.espgpu_set_tuning(drv.ctx, b"gcm_lanes", request.param) == 0
    try:
        yield request.param
    finally:
        drv.lib.espgpu_set_tuning(drv.ctx, b"gcm_lanes", 0)
