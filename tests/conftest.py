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


_GCM_DESIGNS = [((4, 0), "lanes4"), ((8, 0), "lanes8"), ((8, 1 << 30), "burst")]


@pytest.fixture(params=[d for d, _ in _GCM_DESIGNS], ids=[i for _, i in _GCM_DESIGNS])
def gcm_lanes(request, drv):
    """Run a GCM test through every shipped GCM kernel design whatever its
    batch size: the fused kernel with 4 lanes per record (throughput) and
    with 8 (small batches, half the serial steps), and the burst kernel (both
    passes in one launch; decrypt in place keeps the fused kernel).
    set_tuning "gcm_lanes" / "gcm_burst", reset afterwards."""
    lanes, burst = request.param
    assert drv.lib.espgpu_set_tuning(drv.ctx, b"gcm_lanes", lanes) == 0
    assert drv.lib.espgpu_set_tuning(drv.ctx, b"gcm_burst", burst) == 0
    try:
        yield lanes
    finally:
        drv.lib.espgpu_set_tuning(drv.ctx, b"gcm_lanes", 0)
        drv.lib.espgpu_set_tuning(drv.ctx, b"gcm_burst", 4096)
