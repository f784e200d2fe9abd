"""CPU self-tests of table math and circuits the GCM kernel depends on:
* bitsliced AES tail (f-stack_amd/csrc/bsaes.h, compiled into esp_gcm.hip's
  aes_ctr2): the Boyar-Peralta S-box circuit on all 256 inputs, and T-table
  rounds + bitsliced last KR rounds (KR = 1..4) against FIPS-197
  AES-128/192/256 on random blocks;
* GHASH tables (host_crypto.cpp ghash_tables) as the kernel indexes them."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bsaes_selftest(tmp_path):
    exe = tmp_path / "bsaes_selftest"
    csrc = os.path.join(ROOT, "f-stack_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", csrc, "-o", str(exe),
                    os.path.join(ROOT, "tools", "bsaes_selftest.cpp"),
                    os.path.join(csrc, "host_crypto.cpp")], check=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "OK" in r.stdout


def test_ghash_table_layout_selftest(tmp_path):
    """The 8-bit H^8 (LDS) and 4-bit H^1..H^8 (global) GHASH tables the GCM
    kernel indexes, and its stride-8 Horner + final H^(8-l) combination,
    against gf128_mul and a serial GHASH (tools/ghash_selftest.cpp)."""
    import re
    hdr = open(os.path.join(ROOT, "f-stack_amd", "csrc", "espgpu_internal.h")).read()
    # the self-test mirrors these constants; keep them in step with the header
    assert re.search(r"kGh8Bytes = 16 \* 256 \* 16;", hdr)
    assert re.search(r"kGhPowerBytes = 32 \* 16 \* 16;", hdr)
    assert re.search(r"kGh4Off = kGh8Bytes;", hdr)
    assert re.search(r"kGh16Off = kGh4Off \+ 8 \* kGhPowerBytes;", hdr)
    assert re.search(r"kGhTableBytes = kGh16Off \+ kGhPowerBytes;", hdr)
    exe = tmp_path / "ghash_selftest"
    csrc = os.path.join(ROOT, "f-stack_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", csrc, "-o", str(exe),
                    os.path.join(ROOT, "tools", "ghash_selftest.cpp"),
                    os.path.join(csrc, "host_crypto.cpp")], check=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "OK" in r.stdout
