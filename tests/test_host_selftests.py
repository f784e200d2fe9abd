"""CPU self-test of the table math the GCM kernel depends on: the GHASH
tables (host_crypto.cpp ghash_tables) as the kernel indexes them."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_ghash_table_layout_selftest(tmp_path):
    """The 4-bit H^1..H^8 (global) GHASH tables, the 8-bit H^4 and H^8 tables
    the GCM kernels expand from them in LDS (stage_h8_lds / ghash_expand8), and their stride-4 / stride-8 Horner + final
    H^(S-l) combination,
    against gf128_mul and a serial GHASH (tools/ghash_selftest.cpp)."""
    import re
    hdr = open(os.path.join(ROOT, "f-stack_amd", "csrc", "espgpu_internal.h")).read()
    # the self-test mirrors these constants; keep them in step with the header
    assert re.search(r"kGhPowerBytes = 32 \* 16 \* 16;", hdr)
    assert re.search(r"kGh8Bytes = 16 \* 256 \* 16;", hdr)
    assert re.search(r"kGhTableBytes = 8 \* kGhPowerBytes;", hdr)
    assert re.search(r"kGcmLanesPerRec = 4;", hdr) and re.search(r"kGcmLanesSmall = 8;", hdr)
    exe = tmp_path / "ghash_selftest"
    csrc = os.path.join(ROOT, "f-stack_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", csrc, "-o", str(exe),
                    os.path.join(ROOT, "tools", "ghash_selftest.cpp"),
                    os.path.join(csrc, "host_crypto.cpp")], check=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "OK" in r.stdout


def test_bitsliced_aes_selftest(tmp_path):
    """The bitsliced AES the measurement probes run (tools/aes_bs.h: the
    LUT3-packed S-box circuit, key folding, affine constant in the round keys,
    32x32 transposes; tools/bsprobe.hip), built for the CPU with its two
    gfx950 builtins emulated, against host_crypto's table AES for
    AES-128/192/256 counter windows (tools/aes_bs_selftest.cpp)."""
    exe = tmp_path / "aes_bs_selftest"
    csrc = os.path.join(ROOT, "f-stack_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "tools"), "-I", csrc, "-o", str(exe),
                    os.path.join(ROOT, "tools", "aes_bs_selftest.cpp"),
                    os.path.join(csrc, "host_crypto.cpp")], check=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
    assert r.stdout.startswith("OK")


def test_overflow_fifo_arena_selftest(tmp_path):
    """The host overflow's allocator (fifo_arena.h: a bip buffer of
    variable-length allocations, freed oldest first): 200 random alloc / pop
    / undo sequences with wraps against a reference model -- allocations in
    bounds and disjoint, refused exactly when no placement a bip buffer may
    use has room, an emptied arena whole again (tools/fifo_selftest.cpp)."""
    exe = tmp_path / "fifo_selftest"
    csrc = os.path.join(ROOT, "f-stack_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", csrc, "-o", str(exe),
                    os.path.join(ROOT, "tools", "fifo_selftest.cpp")], check=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
    assert r.stdout.startswith("OK")
