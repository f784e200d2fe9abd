"""CPU tests of bench.py's OpenSSL comparison point (tools/ossl_esp.c, the
`cpu_openssl` line; not the reference path): on oracle-encrypted ESP records
it must produce the oracle's plaintext and statuses, so the rate it reports
is for the same work (verify + decrypt of the same records)."""
import os
import sys

import numpy as np
import pytest

from helpers import EtaSA, GcmSA, build_records, oracle_decrypt

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import ossl_esp  # noqa: E402

pytestmark = pytest.mark.skipif(not ossl_esp.available(), reason="tools/libossl_esp.so not built")


def _flip(ct, descs, idx):
    bad = ct.copy()
    for i in idx:
        o = int(descs["off4"][i]) * 4 + int(descs["len"][i]) - 1
        bad[o] ^= 0x40
    return bad


@pytest.mark.parametrize("klen", [16, 32])
def test_openssl_gcm_matches_oracle(klen):
    rng = np.random.default_rng(7 + klen)
    sas = [GcmSA(rng, klen=klen) for _ in range(3)]
    n = 300
    sa_idx = rng.integers(0, 3, n)
    ct_lens = rng.choice([12, 204, 1448, 1449, 8948], n)
    ct_lens = (ct_lens + 3) & ~3
    _, ct, descs, esn = build_records(rng, sas, sa_idx, ct_lens)
    bad = _flip(ct, descs, range(0, n, 7))
    ref, st_ref = oracle_decrypt(sas, bad, descs, esn)
    work = bad.copy()
    t, st = ossl_esp.batch_decrypt("gcm", [s.key for s in sas], work, descs["off4"], descs["len"],
                                   descs["sa"], salts=[s.salt for s in sas], nthreads=4)
    assert t > 0
    assert (st == st_ref).all() and (st[::7] == 74).all() and int((st == 0).sum()) == n - len(range(0, n, 7))
    for i in np.flatnonzero(st == 0):
        o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
        assert work[o + 16:o + L - 16].tobytes() == ref[o + 16:o + L - 16].tobytes()


def test_openssl_cbc_sha1_matches_oracle():
    rng = np.random.default_rng(11)
    sas = [EtaSA(rng, klen=32) for _ in range(4)]
    n = 200
    sa_idx = rng.integers(0, 4, n)
    ct_lens = rng.choice([16, 208, 1440], n)
    _, ct, descs, esn = build_records(rng, sas, sa_idx, ct_lens, gcm=False)
    bad = _flip(ct, descs, range(3, n, 9))
    ref, st_ref = oracle_decrypt(sas, bad, descs, esn)
    work = bad.copy()
    t, st = ossl_esp.batch_decrypt("cbc_sha1", [s.key for s in sas], work, descs["off4"], descs["len"],
                                   descs["sa"], akeys=[s.akey for s in sas], mlen=12, nthreads=3)
    assert t > 0
    assert (st == st_ref).all() and (st[3::9] == 74).all()
    assert (work == ref).all()       # verified records decrypted in place, failed ones untouched


def test_openssl_out_of_place_repeated():
    """The bench's mode: out of place, the sample several times over; the input
    is never written and every pass yields the oracle's plaintext."""
    rng = np.random.default_rng(5)
    sas = [GcmSA(rng) for _ in range(2)]
    n = 64
    sa_idx = rng.integers(0, 2, n)
    _, ct, descs, esn = build_records(rng, sas, sa_idx, np.full(n, 1448))
    ref, st_ref = oracle_decrypt(sas, ct, descs, esn)
    src = ct.copy()
    out = np.zeros_like(ct)
    t, st = ossl_esp.batch_decrypt("gcm", [s.key for s in sas], src, descs["off4"], descs["len"], descs["sa"],
                                   salts=[s.salt for s in sas], nthreads=2, out=out, reps=3)
    assert t > 0 and (st == 0).all() and (st_ref == 0).all()
    assert (src == ct).all()
    for i in range(n):
        o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
        assert out[o + 16:o + L - 16].tobytes() == ref[o + 16:o + L - 16].tobytes()
