"""Helpers for the golden-image fixtures (tests/golden/make_golden_images.py)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def read_pfm(path):
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = (int(x) for x in f.readline().split())
        assert float(f.readline()) < 0
        return np.frombuffer(f.read(), "<f4").reshape(h, w, 3).astype(np.float64)


def cornell64():
    return read_pfm(os.path.join(GOLDEN, "cornell_64x64_16384spp.pfm"))


def cornell256_blocks():
    d = json.load(open(os.path.join(GOLDEN, "cornell_256x256_1024spp_blocks.json")))
    return np.array(d["block_means"]), d["block"]


def veach96():
    return read_pfm(os.path.join(GOLDEN, "veach_96x64_1024spp.pfm"))


def blocks(img, b):
    h, w, _ = img.shape
    return np.asarray(img, np.float64).reshape(h // b, b, w // b, b, 3).mean(axis=(1, 3))


def block_rel(img, ref_blocks, b):
    """Per-block |mean - golden| / (golden + 0.01)."""
    return np.abs(blocks(img, b) - ref_blocks) / (ref_blocks + 1e-2)
