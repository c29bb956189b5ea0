"""Regenerate the committed golden fixtures (run in the BUILD container only).

1. criteo_train_1w.txt.gz — the reference's bundled Criteo sample
   (algorithm/data/criteo/train_1w.txt, 10,000 rows), gzipped: a data file.
2. criteo_ref.npz — outputs of the REFERENCE's own input producer
   (algorithm/deep_learning/utils/dataset.py, imported from /root/reference;
   pandas/sklearn only, TF not needed) under np.random.seed(0):
     create_criteo_dataset('DeepFM', ..., test_size=0.3) -> X_train[:256], y_train[:256]
     create_criteo_dataset('fm', ...)  -> X_train[:256] in compact form
        (dense 13 + the 26 one-hot column indices) and the one-hot width
     features_dict(...)                -> the 26 feat_onehot_dim values
   This pins recommender_system_amd.dataset (a2) against the reference itself.
3. golden_layers.npz / golden_models.npz — fp64 oracle outputs (the
   restatement of the TF graph; parity unpinned by the reference, which has no
   tests and whose TF is not installed) on seeded inputs/weights, incl. FM and
   DeepFM on the bundled sample (config 1).  They freeze the oracle and give
   the GPU tests fixed vectors.

Nothing here is shipped to the GPU box except the .npz/.gz data it writes.
"""
import gzip
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
REF = "/root/reference/algorithm/deep_learning"
SAMPLE = "/root/reference/algorithm/data/criteo/train_1w.txt"

from oracle import ctr_oracle as O  # noqa: E402


def reference_dataset_fixture():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from utils import dataset as ref_ds  # the reference's own module (pandas/sklearn)
    out = {}
    np.random.seed(0)
    (Xtr, ytr), (Xte, yte) = ref_ds.create_criteo_dataset("DeepFM", SAMPLE, test_size=0.3)
    out["deepfm_X_train"] = np.asarray(Xtr[:256], np.float64)
    out["deepfm_y_train"] = np.asarray(ytr[:256], np.int64)
    out["deepfm_n_train"] = np.int64(len(Xtr))
    np.random.seed(0)
    (Ftr, fytr), _ = ref_ds.create_criteo_dataset("fm", SAMPLE, test_size=0.3)
    F = np.asarray(Ftr[:256]).astype(np.float64)
    out["fm_width"] = np.int64(F.shape[1])
    out["fm_dense"] = F[:, :13]
    onehot = F[:, 13:]
    cols = np.stack([np.flatnonzero(r) for r in onehot])  # exactly 26 ones per row
    assert cols.shape[1] == 26 and np.all(onehot.sum(1) == 26)
    out["fm_onehot_cols"] = cols.astype(np.int64)
    out["fm_y_train"] = np.asarray(fytr[:256], np.int64)
    fd = ref_ds.features_dict(SAMPLE)
    out["vocab"] = np.array([f["feat_onehot_dim"] for f in fd[1]], np.int64)
    out["n_dense_cols"] = np.int64(len(fd[0]))
    return out


def layer_fixtures(rng):
    g = {}
    # FM (DeepFM shape, d = 13 + 26*16 = 429, k_fm = 10) and the dense FMLayer
    B, d, kfm = 64, 429, 10
    x = rng.random((B, d)).astype(np.float32)
    w1 = (rng.standard_normal((d, 1)) * 0.05).astype(np.float32)
    v = (rng.standard_normal((d, kfm)) * 0.05).astype(np.float32)
    w0 = np.array([0.01], np.float32)
    g.update(fm_x=x, fm_w0=w0, fm_w1=w1, fm_v=v, fm_out=O.fm_layer(x, w0, w1, v))
    # CrossLayer depth 3
    xc = (rng.standard_normal((B, d)) * 0.3).astype(np.float32)
    ws = (rng.standard_normal((3, d)) * 0.05).astype(np.float32)
    bs = (rng.standard_normal((3, d)) * 0.05).astype(np.float32)
    g.update(cross_x=xc, cross_w=ws, cross_b=bs, cross_out=O.cross_layer(xc, list(ws), list(bs)))
    # InnerProduct [B, 26, 16]
    e = rng.standard_normal((B, 26, 16)).astype(np.float32)
    g.update(inner_e=e, inner_out=O.inner_product_layer(e))
    # DIN attention, prelu, T=100, k=8, (80,40), with an all-masked row
    Ba, T, k = 16, 100, 8
    q = rng.standard_normal((Ba, k)).astype(np.float32)
    key = rng.standard_normal((Ba, T, k)).astype(np.float32)
    lens = rng.integers(0, T + 1, Ba)
    lens[0] = 0
    mask = (np.arange(T)[None] < lens[:, None]).astype(np.float32)
    W1 = rng.uniform(-0.2, 0.2, (4 * k, 80)).astype(np.float32)
    b1 = rng.uniform(-0.1, 0.1, 80).astype(np.float32)
    a1 = rng.uniform(-0.5, 0.5, (T, 80)).astype(np.float32)
    W2 = rng.uniform(-0.2, 0.2, (80, 40)).astype(np.float32)
    b2 = rng.uniform(-0.1, 0.1, 40).astype(np.float32)
    a2 = rng.uniform(-0.5, 0.5, (T, 40)).astype(np.float32)
    W3 = rng.uniform(-0.3, 0.3, (40, 1)).astype(np.float32)
    b3 = np.array([0.02], np.float32)
    p = {"prelu": [(W1, b1, a1), (W2, b2, a2)], "out": (W3, b3)}
    g.update(att_q=q, att_key=key, att_mask=mask, att_W1=W1, att_b1=b1, att_a1=a1, att_W2=W2, att_b2=b2,
             att_a2=a2, att_W3=W3, att_b3=b3, att_out=O.attention(q, key, key, mask, p, "prelu"))
    # DNN tower 429-256-128-64-1 relu
    hid = [(rng.uniform(-0.1, 0.1, (i, o)).astype(np.float32), rng.uniform(-0.05, 0.05, o).astype(np.float32))
           for i, o in ((d, 256), (256, 128), (128, 64))]
    out = (rng.uniform(-0.1, 0.1, (64, 1)).astype(np.float32), np.array([0.03], np.float32))
    for i, (kk, bb) in enumerate(hid):
        g[f"dnn_k{i}"], g[f"dnn_b{i}"] = kk, bb
    g["dnn_kout"], g["dnn_bout"] = out
    g["dnn_out"] = O.dnn_layer(x, hid, out)
    return g


def model_fixtures(rng, ref):
    """Config 1: FM (k=8) and DeepFM (embed 8, k_fm 10) on the bundled sample."""
    g = {}
    width = int(ref["fm_width"])
    dense, cols = ref["fm_dense"], ref["fm_onehot_cols"]
    X = np.zeros((dense.shape[0], width))
    X[:, :13] = dense
    X[np.arange(len(X))[:, None], 13 + cols] = 1.0
    w1 = (rng.standard_normal((width, 1)) * 0.05).astype(np.float32)
    v = (rng.standard_normal((width, 8)) * 0.05).astype(np.float32)
    w0 = np.zeros(1, np.float32)
    g.update(fm_w1=w1, fm_v=v, fm_w0=w0, fm_out=O.fm_model(X, {"w0": w0, "w1": w1, "v": v}))
    Xd = ref["deepfm_X_train"]
    vocab = ref["vocab"]
    tables = [rng.uniform(-0.05, 0.05, (int(n), 8)).astype(np.float32) for n in vocab]
    d = 13 + 26 * 8
    p = {"tables": tables, "w0": np.zeros(1, np.float32),
         "w1": (rng.standard_normal((d, 1)) * 0.05).astype(np.float32),
         "v": (rng.standard_normal((d, 10)) * 0.05).astype(np.float32),
         "dnn_hidden": [(rng.uniform(-0.1, 0.1, (i, o)).astype(np.float32), np.zeros(o, np.float32))
                        for i, o in ((d, 256), (256, 128), (128, 64))],
         "dnn_out": (rng.uniform(-0.1, 0.1, (64, 1)).astype(np.float32), np.zeros(1, np.float32))}
    y, fm, x = O.deepfm(Xd, p)
    g["deepfm_table"] = np.concatenate(tables)
    g.update(deepfm_w0=p["w0"], deepfm_w1=p["w1"], deepfm_v=p["v"], deepfm_out=y, deepfm_fm=fm)
    for i, (kk, bb) in enumerate(p["dnn_hidden"]):
        g[f"deepfm_k{i}"], g[f"deepfm_b{i}"] = kk, bb
    g["deepfm_kout"], g["deepfm_bout"] = p["dnn_out"]
    return g


def main():
    with open(SAMPLE, "rb") as f, gzip.open(os.path.join(HERE, "criteo_train_1w.txt.gz"), "wb", 9) as g:
        shutil.copyfileobj(f, g)
    ref = reference_dataset_fixture()
    np.savez_compressed(os.path.join(HERE, "criteo_ref.npz"), **ref)
    rng = np.random.default_rng(20261015)
    np.savez_compressed(os.path.join(HERE, "golden_layers.npz"), **layer_fixtures(rng))
    np.savez_compressed(os.path.join(HERE, "golden_models.npz"), **model_fixtures(rng, ref))
    for n in os.listdir(HERE):
        print(n, os.path.getsize(os.path.join(HERE, n)))


if __name__ == "__main__":
    main()
