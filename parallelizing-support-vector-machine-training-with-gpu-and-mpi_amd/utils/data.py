"""L0/L1 data layer: CSV datasets, MNIST-shaped synthetic data, min-max scaling.

``load_csv`` mirrors ``read_CSV`` (main3.cpp:13-54, row-limited gpu_svm_main4.cu:16-59) through
the native parser; ``MinMaxScaler`` mirrors ``find_min_max``/``scale_features`` (main3.cpp:57-89)
including the ``range < 1e-12 -> 1`` rule.  ``synthetic_mnist`` produces a deterministic
MNIST-shaped problem (784 integer pixels, digit labels 0-9) because the reference's MNIST CSVs are
not part of the reference repository.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

from .. import _native as N

MNIST_D = 784


@dataclass
class Dataset:
    X: np.ndarray  # (n, d) float64 (or uint8 after compact()), C-contiguous
    y: np.ndarray  # (n,) int32 in {+1, -1}
    labels: np.ndarray  # (n,) int32 raw labels

    @property
    def n(self) -> int:
        return int(self.X.shape[0])

    @property
    def d(self) -> int:
        return int(self.X.shape[1])

    def subset(self, start: int, stop: int) -> "Dataset":
        return Dataset(self.X[start:stop], self.y[start:stop], self.labels[start:stop])

    def compact(self) -> "Dataset":
        """The same dataset with uint8 rows when every feature is an integer in [0, 255] (pixels)."""
        Xc = compact_pixels(self.X)
        return self if (Xc is None or Xc is self.X) else Dataset(Xc, self.y, self.labels)


def compact_pixels(X: np.ndarray) -> Optional[np.ndarray]:
    """uint8 copy of X if every value is an integer in [0, 255], else None.

    MNIST-style pixel data are bytes; the reference holds them as FP64 (read_CSV, main3.cpp:13-54)
    and ships 8 bytes per pixel to the GPU.  The device path accepts the uint8 rows directly and
    widens them to FP64 on the device, where every value is exact, so results are unchanged."""
    X = np.asarray(X)
    if X.dtype == np.uint8:
        return X
    if X.size == 0:
        return None
    if X.dtype.kind == "f" and not np.isfinite(X).all():
        return None
    if X.min() < 0 or X.max() > 255:
        return None
    Xc = X.astype(np.uint8)
    return Xc if np.array_equal(Xc, X) else None


def check_labels(y, n: int) -> np.ndarray:
    """y as int32 of shape (n,) with every label +1 or -1 (main3.cpp:49-52 maps the digit labels);
    ValueError otherwise.  A 0 label falls in neither I_high nor I_low, so a solve would 'converge'
    to a wrong model instead of failing."""
    y = np.ascontiguousarray(y)
    if y.shape != (n,):
        raise ValueError(f"y must have shape ({n},), got {y.shape}")
    if not np.all(np.abs(y) == 1):
        raise ValueError("labels must be +1/-1 (use svm355.utils.data.one_vs_rest)")
    return y.astype(np.int32, copy=False)


def check_warm_start(alpha0, y: np.ndarray, C: float) -> np.ndarray:
    """alpha0 as float64 (n,) that is a feasible point of the dual: finite, inside the box [0, C] (to rounding) and on
    the equality constraint sum(alpha y) = 0 (to rounding).  ValueError otherwise: the solvers assume a
    feasible start, and from an infeasible one they stop on a "converged" model that is not a solution."""
    a = np.ascontiguousarray(alpha0, dtype=np.float64)
    n = y.shape[0]
    if a.shape != (n,):
        raise ValueError(f"alpha0 must have shape ({n},), got {a.shape}")
    # the solvers' own alphas may sit a few ulps outside the box (a_i moves by the rounded step of a_j,
    # as in the reference's update, gpu_svm_main3.cu:441-448): a previous solution must stay a valid start
    tol = 1e-9 * max(1.0, C)
    if not np.all(np.isfinite(a)) or a.min(initial=0.0) < -tol or a.max(initial=0.0) > C + tol:
        raise ValueError(f"alpha0 must be finite and inside [0, C = {C}]")
    s = float(np.dot(a, y.astype(np.float64)))
    if abs(s) > 1e-9 * max(1.0, float(a.sum())):
        raise ValueError(f"alpha0 must satisfy sum(alpha0 * y) = 0 (the dual's equality constraint), got {s:.3g}")
    return a


def check_finite_bounds(mn, mx) -> None:
    """ValueError when a column's min / max is NaN or infinite, i.e. the rows hold a NaN or an infinity
    (numpy's and the device's column bounds propagate NaN): a fit would otherwise find no violating pair
    and return an empty model without saying why."""
    bounds = np.concatenate([np.asarray(mn, dtype=np.float64).ravel(), np.asarray(mx, dtype=np.float64).ravel()])
    if not np.all(np.isfinite(bounds)):
        d = np.asarray(mn).size
        bad = sorted({int(j) for j in np.flatnonzero(~np.isfinite(bounds)) % max(d, 1)})[:8]
        raise ValueError(f"X holds NaN or infinite values (columns {bad}{' ...' if len(bad) == 8 else ''})")


def pixel_rows(X, what: str) -> np.ndarray:
    """X as C-contiguous uint8 (n, d) when every value is an integer in [0, 255]; ValueError naming
    `what` otherwise (never a silent cast: 3.7 or 300 would be truncated or wrapped)."""
    Xc = compact_pixels(X)
    if Xc is None or Xc.ndim != 2:
        raise ValueError(f"{what} needs integer pixel rows (n, d) in [0, 255] (the exact-integer kernel values)")
    return np.ascontiguousarray(Xc)


def one_vs_rest(labels: np.ndarray, positive_label: int = 1) -> np.ndarray:
    """label == positive_label -> +1, else -1 (main3.cpp:49-52 with positive_label = 1)."""
    return np.where(np.asarray(labels) == positive_label, 1, -1).astype(np.int32)


def load_csv(path: str | os.PathLike, limit: Optional[int] = None, positive_label: int = 1,
             n_threads: int = 0) -> Dataset:
    lib = N.core()
    h = lib.svm_csv_load(os.fsencode(str(path)), -1 if limit is None else int(limit), int(positive_label),
                         int(n_threads))
    if not h:
        raise FileNotFoundError(N.last_error())
    try:
        n, d = ctypes.c_int64(), ctypes.c_int64()
        N.check(lib.svm_dataset_dims(h, ctypes.byref(n), ctypes.byref(d)), "svm_dataset_dims")
        X = np.empty((n.value, d.value), dtype=np.float64)
        y = np.empty(n.value, dtype=np.int32)
        lab = np.empty(n.value, dtype=np.int32)
        N.check(lib.svm_dataset_copy(h, N.ptr(X), N.ptr(y), N.ptr(lab)), "svm_dataset_copy")
    finally:
        lib.svm_dataset_free(h)
    return Dataset(X, y, lab)


def write_csv(path: str | os.PathLike, X: np.ndarray, labels: np.ndarray) -> None:
    X = np.ascontiguousarray(X, dtype=np.float64)
    labels = np.ascontiguousarray(labels, dtype=np.int32)
    N.check(N.core().svm_csv_write(os.fsencode(str(path)), N.ptr(X), N.ptr(labels), X.shape[0], X.shape[1]),
            "svm_csv_write")


def synthetic_mnist(n: int, seed: int = 2024, offset: int = 0, positive_label: int = 1,
                    n_threads: int = 0) -> Dataset:
    """Rows [offset, offset + n) of the deterministic MNIST-shaped generator (see csrc/core/synth.cpp).

    Row i depends only on (seed, i): a train split [0, N) and a test split [N, N + M) are disjoint
    draws of the same distribution, and any rank can generate exactly its own partition.
    """
    X = np.empty((n, MNIST_D), dtype=np.float64)
    lab = np.empty(n, dtype=np.int32)
    N.check(N.core().svm_synth_mnist(int(seed), int(offset), int(n), N.ptr(X), N.ptr(lab), int(n_threads)),
            "svm_synth_mnist")
    return Dataset(X, one_vs_rest(lab, positive_label), lab)


class MinMaxScaler:
    """Column min-max scaling to [0, 1] with the reference's degenerate-range rule."""

    def __init__(self, min_: Optional[np.ndarray] = None, max_: Optional[np.ndarray] = None):
        self.min_ = min_
        self.max_ = max_

    def fit(self, X: np.ndarray) -> "MinMaxScaler":
        X = np.ascontiguousarray(X, dtype=np.float64)
        self.min_ = np.empty(X.shape[1])
        self.max_ = np.empty(X.shape[1])
        N.check(N.core().svm_minmax(N.ptr(X), X.shape[0], X.shape[1], N.ptr(self.min_), N.ptr(self.max_)),
                "svm_minmax")
        return self

    def transform(self, X: np.ndarray, copy: bool = True) -> np.ndarray:
        X = np.array(X, dtype=np.float64, order="C", copy=copy)
        if X.shape[0]:
            N.check(N.core().svm_scale(N.ptr(X), X.shape[0], X.shape[1], N.ptr(self.min_), N.ptr(self.max_)),
                    "svm_scale")
        return X

    def fit_transform(self, X: np.ndarray) -> np.ndarray:
        return self.fit(X).transform(X)
