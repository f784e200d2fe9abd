"""Shared test fixtures: synthetic ESP records built and checked with the oracle."""
import json
import os

import numpy as np
import pytest

import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


DESC = np.dtype([("off4", "<u4"), ("len", "<u2"), ("sa", "<u2"), ("esn_hi", "<u4"),
                 ("salt", "<u4")])


class GcmSA:
    def __init__(self, rng, klen=16, esn=False, spi=None, mlen=16):
        self.key = rng.integers(0, 256, klen, dtype=np.uint8).tobytes()
        self.salt = rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
        self.spi = int(rng.integers(256, 2**32 - 1)) if spi is None else spi
        self.esn = esn
        self.mlen = mlen                # ICV bytes: 16, or 12 / 8 truncated (RFC 4106 s3.3)
        self.hlen = 16
        self.oracle = O.SA(O.CSP_MODE_AEAD, self.key, self.salt, mlen=mlen,
                           flags=O.CSP_F_SEPARATE_AAD if esn else 0)

    def esp_sa(self):
        from espgpu.esp import GCM, SecAssoc
        return SecAssoc(self.spi, GCM, self.key + self.salt, esn=self.esn, mlen=self.mlen)


class EtaSA:
    """An encrypt-then-MAC SA: AES-CBC (hlen 24), AES-CTR (RFC 3686, hlen 16,
    salt = the nonce) or ESP-NULL (null=True: CRYPTO_NULL_CBC, no key, no IV,
    hlen 8) with HMAC-SHA1-96 or HMAC-SHA2-256/384/512 (ICV = hashsize/2,
    RFC 4868).  sha: 1, 256, 384 or 512 (sha256=True = 256).  noauth=True:
    the cipher alone (esp_init's CSP_MODE_CIPHER, no ICV)."""

    _AALG = {1: O.CRYPTO_SHA1_HMAC, 256: O.CRYPTO_SHA2_256_HMAC, 384: O.CRYPTO_SHA2_384_HMAC,
             512: O.CRYPTO_SHA2_512_HMAC}
    _MLEN = {1: 12, 256: 16, 384: 24, 512: 32}

    def __init__(self, rng, klen=32, esn=False, spi=None, ctr=False, sha256=False, sha=None, aklen=None,
                 null=False, noauth=False, mlen=None):
        self.noauth, self.null = noauth, null
        self.sha = None if noauth else sha if sha is not None else (256 if sha256 else 1)
        self.key = b"" if null else rng.integers(0, 256, klen, dtype=np.uint8).tobytes()
        if aklen is None:
            aklen = {None: 0, 1: 20, 256: 32, 384: 48, 512: 64}[self.sha]
        self.akey = rng.integers(0, 256, aklen, dtype=np.uint8).tobytes()
        self.ctr, self.sha256 = ctr, self.sha == 256
        self.salt = rng.integers(0, 256, 4, dtype=np.uint8).tobytes() if ctr else b"\0\0\0\0"
        self.spi = int(rng.integers(256, 2**32 - 1)) if spi is None else spi
        self.esn = esn and not noauth
        self.mlen = 0 if noauth else mlen if mlen is not None else self._MLEN[self.sha]
        self.hlen = 16 if ctr else 8 if null else 24
        calg = O.CRYPTO_AES_ICM if ctr else O.CRYPTO_NULL_CBC if null else O.CRYPTO_AES_CBC
        self.oracle = O.SA(O.CSP_MODE_CIPHER if noauth else O.CSP_MODE_ETA, self.key, self.salt,
                           akey=self.akey, mlen=self.mlen, calg=calg,
                           aalg=0 if noauth else self._AALG[self.sha],
                           flags=O.CSP_F_ESN if self.esn else 0)

    def esp_sa(self):
        from espgpu import esp as E
        alg = {("cbc", 1): E.CBC_SHA1, ("cbc", 256): E.CBC_SHA256, ("cbc", 384): E.CBC_SHA384,
               ("cbc", 512): E.CBC_SHA512, ("ctr", 1): E.CTR_SHA1, ("ctr", 256): E.CTR_SHA256,
               ("ctr", 384): E.CTR_SHA384, ("ctr", 512): E.CTR_SHA512, ("null", 1): E.NULL_SHA1,
               ("null", 256): E.NULL_SHA256, ("null", 384): E.NULL_SHA384, ("null", 512): E.NULL_SHA512,
               ("cbc", None): E.CBC, ("ctr", None): E.CTR}
        kind = "ctr" if self.ctr else "null" if self.null else "cbc"
        return E.SecAssoc(self.spi, alg[(kind, self.sha)],
                          self.key + (self.salt if self.ctr else b""), self.akey, esn=self.esn, mlen=self.mlen)


def build_records(rng, sas, sa_idx, ct_lens, gcm=True, stride_pad=0, esn_hi=None, tails=None, seqs=None):
    """Plaintext ESP records + oracle-encrypted copies in one arena.

    Returns (arena_plain, arena_ct, descs, esn_hi) as numpy arrays; records are
    placed at 4-byte aligned offsets (stride_pad adds slack between records).
    tails: {record index: 3 bytes} forced as the payload's last three bytes
    (last pad byte, pad length, next header).  seqs: the records' sequence
    numbers (default i + 1).
    """
    n = len(sa_idx)
    alens = np.array([sas[s].mlen for s in sa_idx], dtype=np.int64)
    hlens = np.array([sas[s].hlen for s in sa_idx], dtype=np.int64)
    lens = np.array([int(h) + int(c) + int(a) for h, c, a in zip(hlens, ct_lens, alens)], dtype=np.int64)
    offs = np.zeros(n, dtype=np.int64)
    pos = 0
    for i in range(n):
        offs[i] = pos
        pos += ((lens[i] + 3) & ~3) + stride_pad
    arena = np.zeros(pos + 64, dtype=np.uint8)
    if esn_hi is None:
        esn_hi = np.zeros(n, dtype=np.uint32)
    payload = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    for i in range(n):
        sa = sas[sa_idx[i]]
        o, L, alen = offs[i], lens[i], alens[i]
        rec = arena[o:o + L]
        rec[:] = payload[o:o + L]
        rec[0:4] = np.frombuffer(sa.spi.to_bytes(4, "big"), dtype=np.uint8)
        sn = int(i + 1) if seqs is None else int(seqs[i])
        rec[4:8] = np.frombuffer(sn.to_bytes(4, "big"), dtype=np.uint8)
        rec[L - alen:] = 0
        if tails is not None and i in tails:        # last 3 payload bytes
            rec[L - alen - 3:L - alen] = np.frombuffer(bytes(tails[i]), dtype=np.uint8)
    descs = np.zeros(n, dtype=DESC)
    descs["off4"] = offs // 4
    descs["len"] = lens
    descs["sa"] = sa_idx
    descs["esn_hi"] = esn_hi
    descs["salt"] = [int.from_bytes(sas[s].salt, "little") for s in sa_idx]
    plain = arena.copy()
    ct = arena.copy()
    _, _ = O.batch([s.oracle for s in sas], ct, descs["off4"], descs["len"], descs["sa"],
                   esn_hi=esn_hi, nthreads=8, encrypt=True)
    return plain, ct, descs, esn_hi


def oracle_decrypt(sas, arena, descs, esn_hi):
    out = arena.copy()
    _, st = O.batch([s.oracle for s in sas], out, descs["off4"], descs["len"], descs["sa"],
                    esn_hi=esn_hi, nthreads=8)
    return out, st
