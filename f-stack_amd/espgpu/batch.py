"""Device-resident batch path (espgpu_decrypt_batch / espgpu_encrypt_batch).

Records live in a torch.uint8 CUDA tensor (the arena, HBM), one 16-byte
espgpu_desc per record in a second tensor.  torch is plumbing here: device
memory and streams.  All crypto runs in libespgpu.so's HIP kernels.
"""
import numpy as np

from . import _lib as L

DESC_DTYPE = np.dtype([("off4", "<u4"), ("len", "<u2"), ("sa", "<u2"),
                       ("esn_hi", "<u4"), ("salt", "<u4")])
assert DESC_DTYPE.itemsize == 16


def descs_to_tensor(descs, device):
    """numpy structured DESC_DTYPE array -> uint8 CUDA tensor (n*16 bytes)."""
    import torch
    raw = np.ascontiguousarray(descs).view(np.uint8)
    return torch.from_numpy(raw.copy()).to(device)


def _stream_ptr(stream):
    if stream is None:
        return None
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


def decrypt_batch(driver, arena, desc, n, status, out=None, grouped=False, stream=None,
                  trailer=None):
    """Verify+decrypt n records.  out=None -> in place (verify-first two-pass).
    trailer: optional int32/uint32 CUDA tensor of n words receiving the fused
    esp_input_cb trailer checks (espgpu_decrypt_batch_trailer; see
    esp.trailer_word for the bit layout)."""
    for t in (arena, desc, status) + tuple(x for x in (out, trailer) if x is not None):
        assert t.is_cuda and t.is_contiguous()
    outp = out.data_ptr() if out is not None else None
    flags = L.BATCH_GROUPED if grouped else 0
    if trailer is not None:
        assert trailer.numel() >= n and trailer.element_size() == 4
        rc = driver.lib.espgpu_decrypt_batch_trailer(
            driver.ctx, arena.data_ptr(), desc.data_ptr(), n, status.data_ptr(), outp,
            trailer.data_ptr(), flags, _stream_ptr(stream))
    else:
        rc = driver.lib.espgpu_decrypt_batch(
            driver.ctx, arena.data_ptr(), desc.data_ptr(), n, status.data_ptr(), outp, flags,
            _stream_ptr(stream))
    if rc:
        raise RuntimeError("espgpu_decrypt_batch: %s" % driver.last_error())


def decrypt_batch_packed(driver, arena, desc, n, status, out, stride, grouped=False, stream=None):
    """Verify+decrypt n GCM records, record i's plaintext to out[i*stride:]
    (espgpu_decrypt_batch_packed: stride a multiple of 128, out of place)."""
    for t in (arena, desc, status, out):
        assert t.is_cuda and t.is_contiguous()
    assert out.numel() >= n * stride
    rc = driver.lib.espgpu_decrypt_batch_packed(
        driver.ctx, arena.data_ptr(), desc.data_ptr(), n, status.data_ptr(), out.data_ptr(), stride,
        L.BATCH_GROUPED if grouped else 0, _stream_ptr(stream))
    if rc:
        raise RuntimeError("espgpu_decrypt_batch_packed: %s (%d)" % (driver.last_error(), rc))


def encrypt_batch(driver, arena, desc, n, status, grouped=False, stream=None):
    for t in (arena, desc, status):
        assert t.is_cuda and t.is_contiguous()
    rc = driver.lib.espgpu_encrypt_batch(
        driver.ctx, arena.data_ptr(), desc.data_ptr(), n, status.data_ptr(),
        L.BATCH_GROUPED if grouped else 0, _stream_ptr(stream))
    if rc:
        raise RuntimeError("espgpu_encrypt_batch: %s" % driver.last_error())


def decrypt_host(driver, arena, desc, n, status, out, chunk=0, flags=0):
    """Host-to-host pipelined decrypt (espgpu_decrypt_host): arena/desc/status/out
    are pinned CPU tensors (torch .pin_memory()); the engine streams chunks
    through HBM with H2D, kernels and D2H overlapped on three HIP streams."""
    for t in (arena, desc, status, out):
        assert not t.is_cuda and t.is_contiguous() and t.is_pinned()
    rc = driver.lib.espgpu_decrypt_host(
        driver.ctx, arena.data_ptr(), arena.numel(), desc.data_ptr(), n, status.data_ptr(),
        out.data_ptr(), chunk, flags)
    if rc:
        raise RuntimeError("espgpu_decrypt_host: %s" % driver.last_error())


REPLAY_DTYPE = np.dtype([("last", "<u8"), ("wsize", "<u4"), ("bitmap_size", "<u4"),
                         ("bitmap_off", "<u4"), ("flags", "<u4")])
assert REPLAY_DTYPE.itemsize == 24


def replay_check(driver, arena, desc, n, replay, bitmap, rstatus, stream=None):
    """Replay pre-filter (espgpu_replay_check_batch): replay is a uint8 CUDA
    tensor of REPLAY_DTYPE records indexed by session id, bitmap an int32 CUDA
    tensor of window words; rstatus receives 0 / EACCES per record, and desc
    is updated in place (len 0 for replayed records, esn_hi for ESN SAs)."""
    for t in (arena, desc, replay, bitmap, rstatus):
        assert t.is_cuda and t.is_contiguous()
    nrep = replay.numel() // REPLAY_DTYPE.itemsize
    rc = driver.lib.espgpu_replay_check_batch(
        driver.ctx, arena.data_ptr(), desc.data_ptr(), n, replay.data_ptr(), nrep,
        bitmap.data_ptr(), rstatus.data_ptr(), _stream_ptr(stream))
    if rc:
        raise RuntimeError("espgpu_replay_check_batch: %s" % driver.last_error())


def replay_merge(driver, status, rstatus, n, stream=None):
    rc = driver.lib.espgpu_replay_merge(driver.ctx, status.data_ptr(), rstatus.data_ptr(), n,
                                        _stream_ptr(stream))
    if rc:
        raise RuntimeError("espgpu_replay_merge: %s" % driver.last_error())
