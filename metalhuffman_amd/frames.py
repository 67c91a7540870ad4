"""Deterministic frame generators for the BASELINE configs.

Every generator derives from the reference's own golden asset BigBridge.png
(2048x1536 8-bit gray, the active TEST_IMAGE4 config, Shared/AAPLRenderer.m:744,
Shared/HuffRenderFrame.m:593-613) or from seeded uniform noise, so the statistics
are natural and every code stays within the reference encoder's 16-bit limit.
"""
from __future__ import annotations

import os

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIGBRIDGE_PNG = os.path.join(_ROOT, "tests", "golden", "BigBridge.png")
BIGBRIDGE_SHA256 = "da4067ee26fb77b14258b92a749594a0aa42fcbba6047b92843663604703021e"


def load_gray_png(path: str) -> np.ndarray:
    from PIL import Image  # only for loading the asset; not on the decode path
    im = Image.open(path)
    if im.mode != "L":
        raise ValueError(f"{path}: expected an 8-bit grayscale PNG, got mode {im.mode}")
    return np.array(im, dtype=np.uint8)


def bigbridge() -> np.ndarray:
    """Config 2 frame: BigBridge.png, 2048x1536 (identity load: the PNG is mode L)."""
    return load_gray_png(BIGBRIDGE_PNG)


def mirror_tile(img: np.ndarray, height: int, width: int) -> np.ndarray:
    """Config 3: tile img with alternating mirrors (cols [g, fliplr g, ...], rows
    [r, flipud r, ...]) and crop to height x width: natural statistics, no seams."""
    row = [img if i % 2 == 0 else img[:, ::-1] for i in range(-(-width // img.shape[1]))]
    strip = np.concatenate(row, axis=1)[:, :width]
    col = [strip if i % 2 == 0 else strip[::-1, :] for i in range(-(-height // img.shape[0]))]
    return np.ascontiguousarray(np.concatenate(col, axis=0)[:height])


def block_shuffle(img: np.ndarray, seed: int, block: int = 8) -> np.ndarray:
    """Config 4/5 frame f: img with its 8x8 blocks permuted by default_rng(seed).
    Per-block deltas keep their multiset, so every shuffled frame has the SAME
    canonical table (a genuinely shared table for the RCCL broadcast)."""
    h, w = img.shape
    if h % block or w % block:
        raise ValueError("block_shuffle needs dimensions that are multiples of the block size")
    bh, bw = h // block, w // block
    blocks = img.reshape(bh, block, bw, block).transpose(0, 2, 1, 3).reshape(bh * bw, block, block)
    perm = np.random.default_rng(seed).permutation(bh * bw)
    out = blocks[perm].reshape(bh, bw, block, block).transpose(0, 2, 1, 3).reshape(h, w)
    return np.ascontiguousarray(out)


def uniform_random(height: int, width: int, seed: int = 1234) -> np.ndarray:
    """Stress frame: uniform bytes (8.000 bits/symbol, every code 8 bits, no T2)."""
    return np.random.default_rng(seed).integers(0, 256, size=(height, width), dtype=np.uint8)


def crop(img: np.ndarray, height: int, width: int) -> np.ndarray:
    """Odd sizes (partial edge blocks), e.g. the 777x1001 crop of BigBridge."""
    return np.ascontiguousarray(img[:height, :width])
