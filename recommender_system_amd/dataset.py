"""Criteo input producer — the host-side mirror of the reference's
utils/dataset.py:19-75 (feature-column dicts + preprocessing), plus a compact
encoding for the GPU path.

Reference behaviour kept (pinned by tests/golden fixtures generated from the
reference itself): missing dense -> 0, missing sparse -> '-1', MinMaxScaler
on I1..I13, then per model type either pandas one-hot (``'fm'``, ``'fnn'``) or
sklearn LabelEncoder codes (``'ffm','DeepCrossing','pnn','dcn','DeepFM','nfm'``),
and an (unseeded unless ``random_state`` is given) train_test_split.
``features_dict`` sizes each sparse field as nunique()+1 over the raw column
(the +1 covers the '-1' fill) and records embed_dim.

``criteo_compact`` returns the same information without the 43,604-wide
one-hot matrix: dense [N,13] float64, label-encoded ids [N,26] int64, and the
per-field offsets of the one-hot block, so that X_onehot[n, 13+off[c]+ids[n,c]]
is the field's single 1 (utils/dataset.py:47-48; verified on the bundled
sample in tests/test_dataset.py).
"""
from __future__ import annotations

import numpy as np
import pandas as pd
from sklearn.model_selection import train_test_split
from sklearn.preprocessing import LabelEncoder, MinMaxScaler

criteo_dense_features = [f"I{i}" for i in range(1, 14)]
criteo_sparse_features = [f"C{i}" for i in range(1, 27)]
_COLUMNS = ["label"] + criteo_dense_features + criteo_sparse_features
_LABEL_ENCODED = ("ffm", "DeepCrossing", "pnn", "dcn", "DeepFM", "nfm")


def sparseFeature(feat, feat_onehot_dim, embed_dim):
    return {"feat": feat, "feat_onehot_dim": feat_onehot_dim, "embed_dim": embed_dim}


def denseFeature(feat):
    return {"feat": feat}


def _read(file_path) -> pd.DataFrame:
    return pd.read_csv(file_path, sep="\t", header=None, names=_COLUMNS)


def _clean_scale(frame: pd.DataFrame) -> pd.DataFrame:
    frame[criteo_dense_features] = frame[criteo_dense_features].fillna(0)
    frame[criteo_sparse_features] = frame[criteo_sparse_features].fillna("-1")
    frame[criteo_dense_features] = MinMaxScaler().fit_transform(frame[criteo_dense_features])
    return frame


def _label_encode(frame: pd.DataFrame) -> pd.DataFrame:
    for col in criteo_sparse_features:
        frame[col] = LabelEncoder().fit_transform(frame[col]).astype(int)
    return frame


def create_criteo_dataset(t, file_path, test_size=0.3, random_state=None):
    """utils/dataset.py:36-65.  Returns ((X_train, y_train), (X_test, y_test))."""
    frame = _clean_scale(_read(file_path))
    if t in ("fm", "fnn"):
        frame = pd.get_dummies(frame)
    elif t in _LABEL_ENCODED:
        frame = _label_encode(frame)
    elif t == "WideDeep":
        onehot = pd.get_dummies(frame).drop(["label"], axis=1)
        frame = pd.concat([_label_encode(frame), onehot], axis=1)
    X = frame.drop(["label"], axis=1).values
    y = frame["label"].values
    X_train, X_test, y_train, y_test = train_test_split(X, y, test_size=test_size, random_state=random_state)
    return (X_train, y_train), (X_test, y_test)


def features_dict(file_path, embed_dim=8):
    """utils/dataset.py:69-75."""
    frame = _read(file_path)
    return [[denseFeature(f) for f in criteo_dense_features],
            [sparseFeature(f, frame[f].nunique() + 1, embed_dim) for f in criteo_sparse_features]]


def criteo_compact(file_path):
    """(dense [N,13] f64, ids [N,26] i64, label [N], onehot_offsets [26]) —
    the compact form of both the label-encoded and the one-hot encodings."""
    frame = _clean_scale(_read(file_path))
    ids = np.empty((len(frame), len(criteo_sparse_features)), dtype=np.int64)
    offsets = np.zeros(len(criteo_sparse_features), dtype=np.int64)
    acc = 0
    for c, col in enumerate(criteo_sparse_features):
        enc = LabelEncoder().fit(frame[col])
        ids[:, c] = enc.transform(frame[col])
        offsets[c] = acc
        acc += len(enc.classes_)
    dense = frame[criteo_dense_features].to_numpy(np.float64)
    return dense, ids, frame["label"].to_numpy(), offsets
