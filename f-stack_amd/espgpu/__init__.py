"""espgpu — MI355X-native ESP bulk-crypto engine for F-Stack's IPsec datapath.

A drop-in opencrypto driver (the role of freebsd/opencrypto/cryptosoft.c) whose
per-packet AES-GCM / AES-CBC+HMAC-SHA1 work runs in HIP kernels on gfx950.
"""
from . import _lib  # noqa: F401
from ._lib import lib  # noqa: F401
from .opencrypto import (CryptoFramework, GpuCryptoDriver, crypto_session_params,  # noqa: F401
                         cryptop)
from .esp import CBC_SHA1, GCM, SecAssoc  # noqa: F401

__all__ = ["lib", "CryptoFramework", "GpuCryptoDriver", "crypto_session_params", "cryptop",
           "SecAssoc", "GCM", "CBC_SHA1"]
