"""Shared helpers for the parity tests: golden fixtures, seeded weights, comparisons."""
import os

import numpy as np

from pntf import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def weights():
    return synth.make_weights(0)


def weight_checksum(w):
    return np.array([float(np.sum(np.abs(v.astype(np.float64)))) for v in w.values()])


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def max_rel(a, b, floor):
    """max |a-b| / max(|b|, floor) elementwise."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), floor)))
