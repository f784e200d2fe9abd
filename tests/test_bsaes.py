"""CPU self-test of the bitsliced AES tail (f-stack_amd/csrc/bsaes.h): the
Boyar-Peralta S-box circuit on all 256 inputs and T-table rounds + bitsliced
last KR rounds (KR = 1..4) against FIPS-197 AES-128/192/256 on random blocks.
The same header is compiled into the GCM kernel (esp_gcm.hip, aes_ctr2)."""
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
