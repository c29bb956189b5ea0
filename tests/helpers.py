"""Shared test helpers: tolerance contract and weight plumbing to the oracle.

Tolerance contract, fp32 kernels vs the fp64 oracle:
  * model outputs (post-sigmoid): |a-b| <= 1e-5 * |b|
  * logits / intermediates:       |a-b| <= 1e-5 * max(|b|, rms(b))
    (the FM logit cancels: fp32 itself is ~1e-4 relative off near zero).
"""
import numpy as np

RTOL = 1e-5


def _np(x):
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    return np.asarray(x, np.float64)


def assert_scaled_close(got, ref, rtol=RTOL, what=""):
    got, ref = _np(got), _np(ref)
    assert got.shape == ref.shape, f"{what}: shape {got.shape} != {ref.shape}"
    if ref.size == 0:
        return
    rms = float(np.sqrt(np.mean(ref ** 2)))
    bound = rtol * np.maximum(np.abs(ref), rms) + 1e-30
    err = np.abs(got - ref)
    bad = ~(err <= bound)
    assert not bad.any(), (f"{what}: {int(bad.sum())}/{bad.size} outside tolerance; "
                           f"max scaled err {float(np.max(err / np.maximum(np.abs(ref), rms))):.3e}")


def assert_rel_close(got, ref, rtol=RTOL, what=""):
    got, ref = _np(got), _np(ref)
    assert got.shape == ref.shape, f"{what}: shape {got.shape} != {ref.shape}"
    err = np.abs(got - ref)
    bad = ~(err <= rtol * np.abs(ref) + 1e-30)
    assert not bad.any(), (f"{what}: {int(bad.sum())}/{bad.size} outside rtol {rtol}; "
                           f"max rel err {float(np.max(err / np.maximum(np.abs(ref), 1e-30))):.3e}")


def criteo_columns(vocabs, n_dense=13, embed_dim=8):
    dense = [{"feat": f"I{i + 1}"} for i in range(n_dense)]
    sparse = [{"feat": f"C{i + 1}", "feat_onehot_dim": int(v), "embed_dim": embed_dim} for i, v in enumerate(vocabs)]
    return [dense, sparse]


def random_ids(rng, B, vocabs, dtype=np.int64):
    return np.stack([rng.integers(0, v, size=B) for v in vocabs], 1).astype(dtype)


def tables_of(embed_layer):
    return [embed_layer.field_table(i).detach().cpu().numpy() for i in range(embed_layer.n_fields)]


def dnn_params(dnn):
    hidden = [(l.kernel.detach().cpu().numpy(), l.bias.detach().cpu().numpy()) for l in dnn.hidden_layer]
    out = (dnn.output_layer.kernel.detach().cpu().numpy(), dnn.output_layer.bias.detach().cpu().numpy())
    return hidden, out


def dropout_masks(seed, offset, B, widths, rate):
    """The dropout multipliers a training step draws for its hidden layers
    (models._Dropout / rs_dropout: one offset range per layer, in order), as
    the oracle's generator restates them; returns (masks, next offset)."""
    from oracle import ctr_oracle as O
    masks, off = [], int(offset)
    for h in widths:
        masks.append(O.dropout_multiplier(B, h, rate, seed, off))
        off += (B * h + 3) // 4 * 4
    return masks, off
