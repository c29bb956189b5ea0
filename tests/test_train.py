"""FM training step: rs_fm_train_step == the oracle's
closed-form SGD step of compile_fit's objective (pinned in test_oracle by
finite differences), over several steps, with repeated rows in a batch
(the deterministic scatter-add), bitwise reproducible run to run."""
import numpy as np
import pytest

from oracle import ctr_oracle as O
from tests.helpers import assert_scaled_close

torch = pytest.importorskip("torch")


@pytest.mark.gpu
@pytest.mark.parametrize("B,k,vmax,id_dtype", [(32, 8, 6, np.int32), (200, 16, 40, np.int64), (1, 4, 3, np.int32)])
def test_fm_train_steps_match_oracle(gpu, B, k, vmax, id_dtype):
    from recommender_system_amd import FM
    rng = np.random.default_rng(B + k)
    vocab = rng.integers(1, vmax, 26)   # small vocabs: many repeated rows per batch
    offs = np.concatenate([[0], np.cumsum(vocab)[:-1]])
    m = FM(k, 1e-3, 2e-3, seed=3)
    n = 13 + int(vocab.sum())
    m.fm.build(n)
    w0, w1, v = (m.fm.w0.cpu().numpy().astype(np.float64), m.fm.w1.cpu().numpy().astype(np.float64),
                 m.fm.v.cpu().numpy().astype(np.float64))
    lr = 0.5  # large, so that the update is visible against fp32 rounding
    for step in range(4):
        dense = rng.random((B, 13)).astype(np.float32)
        ids = np.stack([rng.integers(0, v_, B) for v_ in vocab], 1).astype(id_dtype)
        t = rng.integers(0, 2, B).astype(np.float32)
        loss = m.train_step(dense, ids, t, offs, vocab, lr=lr, return_loss=True)
        x = O.onehot_matrix(dense, ids, vocab)
        w0, w1, v, ce = O.fm_train_step(x, t, w0, w1, v, lr, 1e-3, 2e-3)
        assert_scaled_close(loss, ce, what=f"step {step} loss")
        assert_scaled_close(m.fm.w0, w0, what=f"step {step} w0")
        assert_scaled_close(m.fm.w1, w1, what=f"step {step} w1")
        assert_scaled_close(m.fm.v, v, what=f"step {step} v")
    # the trained weights drive the forward kernels (stale packed images dropped)
    y = m(torch.as_tensor(x, dtype=torch.float32, device=gpu))
    assert_scaled_close(y, O.sigmoid(O.fm_layer(x, w0, w1, v)), what="forward after training")


@pytest.mark.gpu
def test_fm_train_is_deterministic(gpu):
    from recommender_system_amd import FM
    rng = np.random.default_rng(5)
    vocab = rng.integers(1, 4, 26)
    offs = np.concatenate([[0], np.cumsum(vocab)[:-1]])
    dense = rng.random((4096, 13)).astype(np.float32)
    ids = np.stack([rng.integers(0, v_, 4096) for v_ in vocab], 1).astype(np.int32)
    t = rng.integers(0, 2, 4096).astype(np.float32)
    outs = []
    for _ in range(2):
        m = FM(8, seed=9)
        m.fm.build(13 + int(vocab.sum()))
        for _ in range(3):
            m.train_step(dense, ids, t, offs, vocab, lr=0.1)
        outs.append(m.fm.v.cpu().numpy())
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.gpu
def test_compile_fit_on_bundled_sample(gpu):
    """compile_fit mirror on the reference's own bundled Criteo sample
    (config 1's data): the training loss falls and the first epoch's SGD
    steps equal the oracle's."""
    import os

    from recommender_system_amd import FM
    from recommender_system_amd.dataset import criteo_compact, features_dict
    from recommender_system_amd.train import compile_fit
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "criteo_train_1w.txt.gz")
    dense, ids, label, _ = criteo_compact(path)
    vocab = [f["feat_onehot_dim"] for f in features_dict(path)[1]]
    N = 640
    m = FM(8, seed=1)
    m.fm.build(13 + int(np.sum(vocab)))
    w0, w1, v = (m.fm.w0.cpu().numpy().astype(np.float64), m.fm.w1.cpu().numpy().astype(np.float64),
                 m.fm.v.cpu().numpy().astype(np.float64))
    hist = compile_fit(m, dense[:N], ids[:N], label[:N], vocab, batch_size=32, epochs=3, sgd=0.01)
    assert hist[-1] < hist[0]
    m2 = FM(8, seed=1)
    m2.fm.build(13 + int(np.sum(vocab)))
    compile_fit(m2, dense[:N], ids[:N], label[:N], vocab, batch_size=32, epochs=1, sgd=0.01)
    d32 = dense[:N].astype(np.float32)
    for r0 in range(0, N, 32):
        x = O.onehot_matrix(d32[r0:r0 + 32], ids[r0:r0 + 32], vocab)
        w0, w1, v, _ = O.fm_train_step(x, label[r0:r0 + 32], w0, w1, v, 0.01, 1e-4, 1e-4)
    assert_scaled_close(m2.fm.v, v, what="epoch-1 v")
    assert_scaled_close(m2.fm.w1, w1, what="epoch-1 w1")
