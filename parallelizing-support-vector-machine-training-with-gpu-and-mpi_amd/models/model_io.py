"""Model persistence.

The reference's (commented-out) model dump writes four text files, one value per line
(mpi_svm_main3.cpp:754-770, mpi_svm_main2.cpp:685-699):
    final_sv_ids.txt  final_sv_labels.txt  final_sv_alphas.txt  final_b.txt
Those are written natively (svm_model_save) with %.17g so they round-trip bit-exactly.  Because
IDs alone cannot reproduce a prediction without the training set, a loadable model additionally
stores the scaled SV rows (``sv_rows.npy``) and the scaler (``scaler.npz``) in numpy's
pickle-free formats, plus ``model.json`` with the hyper-parameters.
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Optional

import numpy as np

from .. import _native as N
from ..utils.config import SVMParams
from ..utils.data import MinMaxScaler


def save_model(directory, ids, labels, alphas, b, sv_rows=None, scaler: Optional[MinMaxScaler] = None,
               params: Optional[SVMParams] = None, meta: Optional[dict] = None) -> None:
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    ids = np.ascontiguousarray(ids, dtype=np.int64)
    labels = np.ascontiguousarray(labels, dtype=np.int32)
    alphas = np.ascontiguousarray(alphas, dtype=np.float64)
    N.check(N.core().svm_model_save(os.fsencode(str(d)), N.ptr(ids), N.ptr(labels), N.ptr(alphas), ids.shape[0],
                                    float(b)), "svm_model_save")
    if sv_rows is not None:
        np.save(d / "sv_rows.npy", np.ascontiguousarray(sv_rows, dtype=np.float64), allow_pickle=False)
    if scaler is not None:
        np.savez(d / "scaler.npz", min=scaler.min_, max=scaler.max_)
    info = {"format": "svm355-model-v1", "n_sv": int(ids.shape[0]), "b": float(b),
            "params": (params or SVMParams()).as_dict(), "meta": meta or {}}
    (d / "model.json").write_text(json.dumps(info, indent=2))


def _read_column(path: Path, dtype):
    text = path.read_text().split()
    return np.array([dtype(t) for t in text], dtype=np.float64 if dtype is float else np.int64)


def load_model(directory) -> dict:
    d = Path(directory)
    ids = _read_column(d / "final_sv_ids.txt", int).astype(np.int64)
    labels = _read_column(d / "final_sv_labels.txt", int).astype(np.int32)
    alphas = _read_column(d / "final_sv_alphas.txt", float)
    b = float((d / "final_b.txt").read_text().split()[0])
    sv_rows = np.load(d / "sv_rows.npy", allow_pickle=False) if (d / "sv_rows.npy").exists() else None
    scaler = None
    if (d / "scaler.npz").exists():
        z = np.load(d / "scaler.npz", allow_pickle=False)
        scaler = MinMaxScaler(z["min"], z["max"])
    params = SVMParams()
    if (d / "model.json").exists():
        info = json.loads((d / "model.json").read_text())
        params = SVMParams(**info.get("params", {}))
    return {"ids": ids, "labels": labels, "alphas": alphas, "b": b, "sv_rows": sv_rows, "scaler": scaler,
            "params": params}
