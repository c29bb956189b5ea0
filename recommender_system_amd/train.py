"""compile_fit on the MI355X path.

Mirror of utils/compile_fit.py:9-15: ``tf.data.Dataset.from_tensor_slices((X,
y)).batch(batch_size)`` (no shuffle: the dataset order), SGD(sgd),
binary cross-entropy, ``epochs`` passes.  The data is the compact form of the
reference's X (dataset.criteo_compact / an RSCB file): dense [N, nd], label
codes [N, F], labels [N], per-field vocab.  Each batch is one
``model.train_step``: ``FM`` (rs_fm_train_step; the one-hot X of
model/fm.py), ``DeepFM`` (model/deepFM.py), ``DCN`` (model/dcn.py), ``NFM``
(model/nfm.py) or ``FFM`` (model/ffm.py) on dense + label-encoded X, and
``DIN`` (model/din.py:106) on the reference's input dict (pass it as
``dense``, ``ids=None``; every value is sliced along its first axis).
"""
from __future__ import annotations

import numpy as np
import torch

from .models import DCN, DIN, FFM, FM, NFM, DeepFM


def compile_fit(model, dense, ids, labels, field_vocab=None, batch_size=32, epochs=10, sgd=0.01, device=None):
    """Train ``model`` (models.FM / DeepFM / DCN / NFM / FFM / DIN) in place;
    returns the per-epoch mean cross-entropy (before each step, without the l2
    terms).  ``field_vocab`` (feat_onehot_dim per field) is needed for FM's
    one-hot layout; the others read it from their layers.  PNN trains with its
    own loop in the reference (model/pnn.py:74-81): PNN.train_step."""
    if not isinstance(model, (FM, DeepFM, DCN, NFM, FFM, DIN)):
        raise NotImplementedError("compile_fit: FM, DeepFM, DCN, NFM, FFM and DIN (PNN: PNN.train_step)")
    dev = torch.device(device) if device is not None else model._dev
    labels = torch.as_tensor(np.asarray(labels, np.float32), device=dev)
    N = labels.shape[0]
    history = []
    if isinstance(model, DIN):
        if ids is not None:
            raise ValueError("compile_fit(DIN): pass the input dict as `dense` and ids=None")
        data = {key: torch.as_tensor(np.asarray(val), device=dev) for key, val in dense.items()}
        for _ in range(epochs):
            losses = [model.train_step({key: val[r0:r0 + batch_size] for key, val in data.items()},
                                       labels[r0:r0 + batch_size], lr=sgd, return_loss=True, check_ids=False)
                      for r0 in range(0, N, batch_size)]
            history.append(float(torch.cat(losses).mean().item()))
        return history
    dense = torch.as_tensor(np.asarray(dense, np.float32), device=dev)
    ids = torch.as_tensor(np.asarray(ids), device=dev)
    if isinstance(model, FM):
        if field_vocab is None:
            raise ValueError("compile_fit(FM): field_vocab is required (the one-hot layout)")
        vocab = np.asarray(field_vocab, np.int64)
        offs = np.concatenate([[0], np.cumsum(vocab)[:-1]])
        step = lambda d, i, t: model.train_step(d, i, t, offs, vocab, lr=sgd, return_loss=True, check_ids=False)
    elif isinstance(model, FFM):
        step = lambda d, i, t: model.train_step((d, i), t, lr=sgd, return_loss=True)
    else:
        step = lambda d, i, t: model.train_step((d, i), t, lr=sgd, return_loss=True, check_ids=False)
    for _ in range(epochs):
        losses = [step(dense[r0:r0 + batch_size], ids[r0:r0 + batch_size], labels[r0:r0 + batch_size])
                  for r0 in range(0, N, batch_size)]
        history.append(float(torch.cat(losses).mean().item()))
    return history
