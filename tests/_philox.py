"""numpy Philox4x32-10 replay of the device dropout streams (test infrastructure).

The HIP kernels draw keep decisions as (csrc/mmf_device.h):
    counter = (idx>>3 lo32, idx>>3 hi32, site, offset lo32), key = (seed lo32, seed hi32)
    word    = philox10(counter, key)[(idx >> 1) & 3]
    keep    = ((word >> 16*(idx & 1)) & 0xFFFF) >= ceil(p * 65536)
so a test can rebuild the exact masks and run the CPU oracle in train mode.
"""
from __future__ import annotations

import numpy as np
import torch

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)


def philox10(c0, c1, c2, c3, k0, k1):
    c0, c1, c2, c3 = (np.asarray(v, dtype=np.uint64) for v in (c0, c1, c2, c3))
    k0, k1 = np.uint64(k0), np.uint64(k1)
    for _ in range(10):
        p0 = _M0 * c0
        p1 = _M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & _MASK, lo1, (hi0 ^ c3 ^ k1) & _MASK, lo0
        k0 = (k0 + _W0) & _MASK
        k1 = (k1 + _W1) & _MASK
    return c0, c1, c2, c3


def keep_mask(shape, site: int, seed: int, offset: int, p: float) -> np.ndarray:
    """8 decisions per Philox call: block idx>>3, word (idx>>1)&3, 16-bit half idx&1;
    keep iff u16 >= ceil(p * 65536) (csrc/mmf_device.h keep1/keep4)."""
    n = int(np.prod(shape))
    nblk = (n + 7) // 8
    blk = np.arange(nblk, dtype=np.uint64)
    words = philox10(blk & _MASK, blk >> np.uint64(32), np.full(nblk, site, np.uint64),
                     np.full(nblk, offset & 0xFFFFFFFF, np.uint64), seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    # one call per 8 elements: element idx takes word (idx >> 1) & 3, half idx & 1 -- the
    # little-endian u16 order of the call's four u32 words
    w32 = np.stack([w.astype(np.uint32) for w in words], axis=1)
    u16 = w32.view("<u2").reshape(-1)[:n]
    thr = np.uint16(int(np.ceil(np.float32(p) * np.float32(65536.0))))
    return (u16 >= thr).reshape(shape)


def mask_provider(seed: int, offset: int, p: float):
    """Callable (site, tensor) -> keep mask for oracle.hybrid_cpu._dropout."""
    def fn(site, x):
        return torch.from_numpy(keep_mask(tuple(x.shape), site, seed, offset, p))
    return fn
