"""SPI-hash sharding of SAs across GPUs (one process per GPU, no collective).

The hash is the one FreeBSD's SADB uses to bucket SAs by SPI:
key_u32hash(spi) = fnv_32_buf(&spi, 4, FNV1_32_INIT)   freebsd/netipsec/key.c:295-299
fnv_32_buf: hval *= FNV_32_PRIME; hval ^= byte        freebsd/sys/fnv_hash.h:23-31
over the SPI as stored in struct secasvar (network byte order).
"""
FNV1_32_INIT = 33554467
FNV_32_PRIME = 0x01000193


def fnv_32_buf(data, hval=FNV1_32_INIT):
    for b in bytes(data):
        hval = (hval * FNV_32_PRIME) & 0xFFFFFFFF
        hval ^= b
    return hval


def key_u32hash(spi):
    """spi as an integer in host order; hashed over its network-order bytes."""
    return fnv_32_buf(int(spi).to_bytes(4, "big"))


def gpu_of_spi(spi, ngpus):
    return key_u32hash(spi) % ngpus


def spis_for_rank(rank, ngpus, count, start=0x100):
    """The first `count` SPIs >= start that hash to `rank` (deterministic)."""
    out, s = [], start
    while len(out) < count:
        if gpu_of_spi(s, ngpus) == rank:
            out.append(s)
        s += 1
    return out


def random_spis(count, seed):
    """`count` distinct random SPIs >= 256 (SPIs 1..255 are reserved, RFC 4303 2.1)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    out = set()
    while len(out) < count:
        out.update(int(x) for x in rng.integers(256, 2**32, count - len(out), dtype=np.uint64))
    return sorted(out)


def shard_plan(spis, sa_of_packet, rank, ngpus):
    """SPI-hash partition of a global batch: (local SA indices, local packet
    indices) owned by `rank`.  Every packet goes where its SA's SPI hashes."""
    import numpy as np
    owner = np.array([gpu_of_spi(s, ngpus) for s in spis], dtype=np.int64)
    local_sas = np.nonzero(owner == rank)[0]
    local_pkts = np.nonzero(owner[np.asarray(sa_of_packet)] == rank)[0]
    return local_sas, local_pkts
