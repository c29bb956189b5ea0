"""compile_fit for the FM model on the MI355X path.

Mirror of utils/compile_fit.py:9-15: ``tf.data.Dataset.from_tensor_slices((X,
y)).batch(batch_size)`` (no shuffle: the dataset order), SGD(sgd),
binary cross-entropy, ``epochs`` passes.  The data is the compact form of the
reference's one-hot X (dataset.criteo_compact / an RSCB file): dense
[N, nd], label codes [N, F], labels [N], per-field vocab.  Each batch is one
``FM.train_step`` (rs_fm_train_step).
"""
from __future__ import annotations

import numpy as np
import torch


def compile_fit(model, dense, ids, labels, field_vocab, batch_size=32, epochs=10, sgd=0.01, device=None):
    """Train ``model`` (models.FM) in place; returns the per-epoch mean
    cross-entropy (before each step, without the l2 terms)."""
    dev = torch.device(device) if device is not None else model._dev
    dense = torch.as_tensor(np.asarray(dense, np.float32), device=dev)
    ids = torch.as_tensor(np.asarray(ids), device=dev)
    labels = torch.as_tensor(np.asarray(labels, np.float32), device=dev)
    vocab = np.asarray(field_vocab, np.int64)
    offs = np.concatenate([[0], np.cumsum(vocab)[:-1]])
    N = dense.shape[0]
    history = []
    for _ in range(epochs):
        losses = []
        for r0 in range(0, N, batch_size):
            r1 = min(N, r0 + batch_size)
            losses.append(model.train_step(dense[r0:r1], ids[r0:r1], labels[r0:r1], offs, vocab, lr=sgd,
                                           return_loss=True, check_ids=False))
        history.append(float(torch.cat(losses).mean().item()))
    return history
