"""CPU: known-answer tests that pin the oracle (the reference has no tests and
its TF/Keras arithmetic cannot run here), plus the oracle's Keras semantics."""
import numpy as np
import pytest

from oracle import ctr_oracle as O


def test_fm_trick_equals_pairwise():
    rng = np.random.default_rng(0)
    x = rng.random((20, 37))
    v = rng.standard_normal((37, 6)) * 0.05
    w1 = rng.standard_normal((37, 1)) * 0.05
    w0 = np.array([0.3])
    a = O.fm_layer(x, w0, w1, v)
    b = O.fm_layer_pairwise(x, w0, w1, v)
    np.testing.assert_allclose(a, b, rtol=0, atol=1e-13)


def test_fm_onehot_equals_gather():
    rng = np.random.default_rng(1)
    vocabs = rng.integers(2, 30, 26)
    offs = np.concatenate([[0], np.cumsum(vocabs)[:-1]])
    B, nd = 17, 13
    ids = np.stack([rng.integers(0, v, B) for v in vocabs], 1)
    dense = rng.random((B, nd))
    n = nd + vocabs.sum()
    x = np.zeros((B, n))
    x[:, :nd] = dense
    x[np.arange(B)[:, None], nd + offs[None] + ids] = 1
    v = rng.standard_normal((n, 8)) * 0.05
    w1 = rng.standard_normal((n, 1)) * 0.05
    w0 = np.array([0.1])
    np.testing.assert_allclose(O.fm_onehot_gather(dense, ids, offs, w0, w1, v), O.fm_layer(x, w0, w1, v),
                               rtol=0, atol=1e-13)


def test_cross_layer_equals_loop():
    rng = np.random.default_rng(2)
    x = rng.standard_normal((9, 21))
    ws = [rng.standard_normal(21) * 0.05 for _ in range(4)]
    bs = [rng.standard_normal(21) * 0.05 for _ in range(4)]
    np.testing.assert_allclose(O.cross_layer(x, ws, bs), O.cross_layer_loop(x, ws, bs), rtol=1e-13, atol=1e-13)


def test_cross_affine_closed_form():
    """x_L = alpha_L x0 + beta_L — the identity the MFMA CrossNet kernel uses."""
    rng = np.random.default_rng(3)
    x = rng.standard_normal((5, 30))
    ws = [rng.standard_normal(30) * 0.1 for _ in range(3)]
    bs = [rng.standard_normal(30) * 0.1 for _ in range(3)]
    beta = np.zeros(30)
    alpha = np.ones(5)
    for w, b in zip(ws, bs):
        g = x @ w
        h = beta @ w
        alpha = alpha * (1 + g) + h
        beta = beta + b
    np.testing.assert_allclose(alpha[:, None] * x + beta, O.cross_layer(x, ws, bs), rtol=1e-12, atol=1e-12)


def test_inner_product_equals_loop_and_order():
    rng = np.random.default_rng(4)
    e = rng.standard_normal((3, 6, 5))
    np.testing.assert_allclose(O.inner_product_layer(e), O.inner_product_loop(e), rtol=1e-13)
    row, col = O.pair_indices(4)
    assert list(zip(row, col)) == [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]


def _att_params(rng, k, T, h=(8, 4)):
    W1 = rng.uniform(-0.3, 0.3, (4 * k, h[0]))
    W2 = rng.uniform(-0.3, 0.3, (h[0], h[1]))
    return {"prelu": [(W1, np.zeros(h[0]), rng.uniform(-.5, .5, (T, h[0]))),
                      (W2, np.zeros(h[1]), rng.uniform(-.5, .5, (T, h[1])))],
            "out": (rng.uniform(-0.3, 0.3, (h[1], 1)), np.zeros(1))}


def test_attention_single_unmasked_and_all_masked():
    rng = np.random.default_rng(5)
    B, T, k = 3, 7, 4
    q = rng.standard_normal((B, k))
    key = rng.standard_normal((B, T, k))
    mask = np.zeros((B, T))
    mask[0, 3] = 1  # one valid position -> that value row
    p = _att_params(rng, k, T)
    out = O.attention(q, key, key, mask, p)
    np.testing.assert_allclose(out[0], key[0, 3], rtol=1e-12)
    np.testing.assert_allclose(out[1], key[1].mean(0), rtol=1e-12)  # fully masked -> uniform


def test_mask_fill_value_is_float32_rounded():
    assert O.MASK_FILL == -4294967295
    assert np.float32(O.MASK_FILL) == np.float32(-4294967296.0)


def test_embedding_cast_and_range():
    t = np.arange(12.0).reshape(6, 2)
    ids = np.array([0.9, 5.99, -0.5])
    np.testing.assert_array_equal(O.embedding_lookup(t, ids), t[[0, 5, 0]])  # truncation toward zero
    with pytest.raises(IndexError):
        O.embedding_lookup(t, np.array([6]))
    with pytest.raises(IndexError):
        O.embedding_lookup(t, np.array([-1.0]))


def test_embed_layer_is_field_major_flat():
    t0 = np.arange(6.0).reshape(3, 2)
    t1 = 10 + np.arange(8.0).reshape(4, 2)
    out = O.embed_layer(np.array([[1, 3], [0, 0]]), [t0, t1])
    np.testing.assert_array_equal(out, [[2, 3, 16, 17], [0, 1, 10, 11]])


def test_dice_and_bn_inference():
    x = np.array([[0.5, -2.0]])
    y = O.dice(x, alpha=np.array([0.25, 0.25]), mean=np.zeros(2), var=np.ones(2), eps=1e-9)
    p = 1 / (1 + np.exp(-x / np.sqrt(1 + 1e-9)))
    np.testing.assert_allclose(y, 0.25 * (1 - p) * x + p * x)
    np.testing.assert_allclose(O.batchnorm_inference(x, 0, 1, eps=1e-3), x / np.sqrt(1.001))


def test_deepfm_oracle_composition():
    rng = np.random.default_rng(6)
    vocabs = [5, 7, 3]
    tables = [rng.uniform(-0.05, 0.05, (v, 4)) for v in vocabs]
    d = 2 + 3 * 4
    p = {"tables": tables, "w0": np.zeros(1), "w1": rng.standard_normal((d, 1)) * 0.05,
         "v": rng.standard_normal((d, 3)) * 0.05,
         "dnn_hidden": [(rng.uniform(-.1, .1, (d, 8)), np.zeros(8))], "dnn_out": (rng.uniform(-.1, .1, (8, 1)), np.zeros(1))}
    X = np.concatenate([rng.random((4, 2)), np.stack([rng.integers(0, v, 4) for v in vocabs], 1)], 1)
    y, fm, x = O.deepfm(X, p, nd=2)
    dnn = O.dnn_layer(x, p["dnn_hidden"], p["dnn_out"])
    np.testing.assert_allclose(y, 1 / (1 + np.exp(-0.5 * (fm + dnn))))


def test_outer_product_equals_loop():
    """OuterProductLayer op-for-op restatement == per-pair e_col . (W_p e_row)."""
    rng = np.random.default_rng(5)
    e = rng.standard_normal((3, 5, 4))
    W = rng.standard_normal((4, 10, 4))
    np.testing.assert_allclose(O.outer_product_layer(e, W), O.outer_product_loop(e, W), rtol=1e-12, atol=1e-12)
    # identity W_p -> plain inner product
    Wi = np.repeat(np.eye(4)[:, None, :], 10, axis=1)
    np.testing.assert_allclose(O.outer_product_layer(e, Wi), O.inner_product_layer(e), rtol=1e-12, atol=1e-12)


def test_fm_train_step_gradient_matches_finite_differences():
    """The closed-form FM training gradient (oracle.fm_train_step, the
    restatement of compile_fit's SGD on FM) == central differences of the
    regularised loss, on a one-hot x with a repeated row."""
    rng = np.random.default_rng(11)
    vocab = [3, 4]
    dense = rng.random((5, 2))
    ids = np.array([[0, 1], [2, 1], [0, 3], [1, 1], [0, 0]])
    x = O.onehot_matrix(dense, ids, vocab)
    t = rng.integers(0, 2, 5).astype(float)
    w0, w1, v = np.array([0.1]), rng.normal(size=(9, 1)), rng.normal(size=(9, 3))
    lr, l2w, l2v = 1.0, 1e-2, 2e-2
    n0, n1, nv, _ = O.fm_train_step(x, t, w0, w1, v, lr, l2w, l2v)
    grads = [(w0 - n0), (w1 - n1), (v - nv)]
    eps = 1e-6
    for p, gp in zip((w0, w1, v), grads):
        for idx in np.ndindex(p.shape):
            keep = p[idx]
            p[idx] = keep + eps
            lp = O.fm_loss(x, t, w0, w1, v, l2w, l2v)[0]
            p[idx] = keep - eps
            lm = O.fm_loss(x, t, w0, w1, v, l2w, l2v)[0]
            p[idx] = keep
            assert abs((lp - lm) / (2 * eps) - gp[idx]) < 1e-7


def test_deepfm_train_step_gradient_matches_finite_differences():
    """oracle.deepfm_train_step's hand backprop == central differences of
    compile_fit's DeepFM objective, for embedding rows (one repeated in the
    batch), DNN weights of every layer, FM w0 / w1 / v."""
    rng = np.random.default_rng(12)
    nd, k, kfm = 2, 3, 2
    vocab = [3, 2]
    tables = [rng.normal(size=(v_, k)) * 0.5 for v_ in vocab]
    d = nd + len(vocab) * k
    p = {"tables": tables, "w0": np.array([0.1]), "w1": rng.normal(size=(d, 1)), "v": rng.normal(size=(d, kfm)),
         "dnn_hidden": [(rng.normal(size=(d, 5)), rng.normal(size=5) * 0.1),
                        (rng.normal(size=(5, 3)), rng.normal(size=3) * 0.1)],
         "dnn_out": (rng.normal(size=(3, 1)), np.array([0.05]))}
    dense = rng.random((4, nd))
    ids = np.array([[0, 1], [2, 1], [0, 0], [1, 1]])
    t = np.array([1.0, 0.0, 1.0, 0.0])
    lr, l2w, l2v = 1.0, 1e-2, 3e-2
    new, _ = O.deepfm_train_step(dense, ids, t, p, lr, l2w, l2v, nd=nd)
    eps = 1e-6

    def check(arr, new_arr, idx):
        keep = arr[idx]
        arr[idx] = keep + eps
        lp = O.deepfm_loss(dense, ids, t, p, l2w, l2v, nd=nd)
        arr[idx] = keep - eps
        lm = O.deepfm_loss(dense, ids, t, p, l2w, l2v, nd=nd)
        arr[idx] = keep
        assert abs((lp - lm) / (2 * eps) - (arr[idx] - new_arr[idx]) / lr) < 1e-6, idx

    for idx in [(0, 0), (0, 2), (2, 1), (1, 0)]:
        check(p["tables"][0], new["tables"][0], idx)
    check(p["tables"][1], new["tables"][1], (1, 2))
    check(p["w0"], new["w0"], (0,))
    for idx in [(0, 0), (5, 0), (7, 0)]:
        check(p["w1"], new["w1"], idx)
    for idx in [(1, 1), (6, 0)]:
        check(p["v"], new["v"], idx)
    for li in range(2):
        for idx in [(0, 0), (2, 1)]:
            check(p["dnn_hidden"][li][0], new["dnn_hidden"][li][0], idx)
        check(p["dnn_hidden"][li][1], new["dnn_hidden"][li][1], (1,))
    check(p["dnn_out"][0], new["dnn_out"][0], (2, 0))
    check(p["dnn_out"][1], new["dnn_out"][1], (0,))


def test_philox_known_answers_and_dropout_multiplier():
    """The dropout generator (rs_dropout / oracle.dropout_multiplier) is
    Philox4x32-10: Random123's known-answer vectors, restated with Python ints
    here, and the vectorised oracle agree; the multiplier keeps ~1 - rate of
    the elements at scale 1/(1-rate), and a draw depends on (seed, offset)."""
    M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85

    def ph(c, k0, k1):
        for _ in range(10):
            p0, p1 = M0 * c[0], M1 * c[2]
            c = [(p1 >> 32) ^ c[1] ^ k0, p1 & 0xFFFFFFFF, (p0 >> 32) ^ c[3] ^ k1, p0 & 0xFFFFFFFF]
            k0, k1 = (k0 + W0) & 0xFFFFFFFF, (k1 + W1) & 0xFFFFFFFF
        return c

    assert ph([0, 0, 0, 0], 0, 0) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert ph([0xFFFFFFFF] * 4, 0xFFFFFFFF, 0xFFFFFFFF) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert ph([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], 0xA4093822, 0x299F31D0) == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]
    seed = (0xBEEF << 32) | 0x1234
    ctr = np.array([0, 1, 2 ** 32 + 5], np.uint64)
    got = O.philox4x32_10(ctr, seed)
    for i, c in enumerate(ctr.tolist()):
        assert got[i].tolist() == ph([c & 0xFFFFFFFF, c >> 32, 0, 0], seed & 0xFFFFFFFF, seed >> 32)
    m = O.dropout_multiplier(512, 300, 0.2, seed, 8)
    assert set(np.unique(m).tolist()) == {0.0, 1.25}
    assert abs(float((m == 0).mean()) - 0.2) < 0.005
    assert not np.array_equal(m, O.dropout_multiplier(512, 300, 0.2, seed, 8 + 4 * 512 * 75))
    np.testing.assert_array_equal(m.reshape(-1)[4:], O.dropout_multiplier(1, 512 * 300 - 4, 0.2, seed, 12)[0])


def test_train_steps_with_dropout_match_finite_differences():
    """deepfm_train_step / dcn_train_step with DNNLayer dropout masks (fixed
    multipliers, as one training step draws them) == central differences of
    the objective with the same masks: the gradient flows through kept units
    scaled by 1/(1-rate) and stops at dropped ones."""
    rng = np.random.default_rng(21)
    nd, k, kfm = 2, 3, 2
    vocab = [3, 2]
    B = 5
    tables = [rng.normal(size=(v_, k)) * 0.5 for v_ in vocab]
    d = nd + len(vocab) * k
    hidden = [(rng.normal(size=(d, 6)), rng.normal(size=6) * 0.1), (rng.normal(size=(6, 4)), rng.normal(size=4) * 0.1)]
    masks = [O.dropout_multiplier(B, 6, 0.3, 77, 0), O.dropout_multiplier(B, 4, 0.3, 77, 32)]
    assert all((mk == 0).any() and (mk > 0).any() for mk in masks)
    dense = rng.random((B, nd))
    ids = np.array([[0, 1], [2, 1], [0, 0], [1, 1], [2, 0]])
    t = np.array([1.0, 0.0, 1.0, 0.0, 1.0])
    eps = 1e-6
    p = {"tables": tables, "w0": np.array([0.1]), "w1": rng.normal(size=(d, 1)), "v": rng.normal(size=(d, kfm)),
         "dnn_hidden": hidden, "dnn_out": (rng.normal(size=(4, 1)), np.array([0.05]))}
    new, _ = O.deepfm_train_step(dense, ids, t, p, 1.0, 1e-2, 3e-2, nd=nd, masks=masks)
    q = {"tables": [tb.copy() for tb in tables], "cross_w": [rng.normal(size=(d, 1)) * 0.3 for _ in range(2)],
         "cross_b": [rng.normal(size=(d, 1)) * 0.3 for _ in range(2)],
         "dnn_hidden": [(W.copy(), b.copy()) for W, b in hidden], "dnn_out": (rng.normal(size=(4, 2)), np.zeros(2)),
         "out_kernel": rng.normal(size=(d + 2, 1)) * 0.3, "out_bias": np.array([0.05])}
    newq, _ = O.dcn_train_step(dense, ids, t, q, 1.0, 1e-2, 3e-2, nd=nd, masks=masks)

    def check(loss, arr, new_arr, idx):
        keep = arr[idx]
        arr[idx] = keep + eps
        lp = loss()
        arr[idx] = keep - eps
        lm = loss()
        arr[idx] = keep
        assert abs((lp - lm) / (2 * eps) - (arr[idx] - new_arr[idx])) < 1e-6, idx

    fl = lambda: O.deepfm_loss(dense, ids, t, p, 1e-2, 3e-2, nd=nd, masks=masks)
    gl = lambda: O.dcn_loss(dense, ids, t, q, 1e-2, 3e-2, nd=nd, masks=masks)
    for li in range(2):
        for idx in [(0, 0), (2, 1), (5, 3)]:
            check(fl, p["dnn_hidden"][li][0], new["dnn_hidden"][li][0], idx)
            check(gl, q["dnn_hidden"][li][0], newq["dnn_hidden"][li][0], idx)
        check(fl, p["dnn_hidden"][li][1], new["dnn_hidden"][li][1], (3,))
    for idx in [(0, 0), (2, 2), (1, 1)]:
        check(fl, p["tables"][0], new["tables"][0], idx)
        check(gl, q["tables"][0], newq["tables"][0], idx)
    check(fl, p["dnn_out"][0], new["dnn_out"][0], (2, 0))
    check(gl, q["dnn_out"][0], newq["dnn_out"][0], (1, 1))


def test_dcn_train_step_gradient_matches_finite_differences():
    """oracle.dcn_train_step's hand backprop (CrossNet delta recursion, DNN,
    output Dense, embedding scatter-add) == central differences of
    compile_fit's DCN objective with CrossLayer's l2 terms."""
    rng = np.random.default_rng(13)
    nd, k, L, od = 2, 3, 3, 2
    vocab = [3, 2]
    tables = [rng.normal(size=(v_, k)) * 0.5 for v_ in vocab]
    d = nd + len(vocab) * k
    p = {"tables": tables,
         "cross_w": [rng.normal(size=(d, 1)) * 0.3 for _ in range(L)],
         "cross_b": [rng.normal(size=(d, 1)) * 0.3 for _ in range(L)],
         "dnn_hidden": [(rng.normal(size=(d, 5)), rng.normal(size=5) * 0.1)],
         "dnn_out": (rng.normal(size=(5, od)), rng.normal(size=od) * 0.1),
         "out_kernel": rng.normal(size=(d + od, 1)) * 0.3, "out_bias": np.array([0.05])}
    dense = rng.random((4, nd))
    ids = np.array([[0, 1], [2, 1], [0, 0], [1, 1]])
    t = np.array([1.0, 0.0, 1.0, 0.0])
    lr, rw, rb = 1.0, 1e-2, 3e-2
    new, _ = O.dcn_train_step(dense, ids, t, p, lr, rw, rb, nd=nd)
    eps = 1e-6

    def check(arr, new_arr, idx):
        keep = arr[idx]
        arr[idx] = keep + eps
        lp = O.dcn_loss(dense, ids, t, p, rw, rb, nd=nd)
        arr[idx] = keep - eps
        lm = O.dcn_loss(dense, ids, t, p, rw, rb, nd=nd)
        arr[idx] = keep
        assert abs((lp - lm) / (2 * eps) - (arr[idx] - new_arr[idx]) / lr) < 1e-6, idx

    for idx in [(0, 0), (0, 2), (2, 1), (1, 0)]:
        check(p["tables"][0], new["tables"][0], idx)
    check(p["tables"][1], new["tables"][1], (1, 2))
    for l in range(L):
        for idx in [(0, 0), (4, 0), (7, 0)]:
            check(p["cross_w"][l], new["cross_w"][l], idx)
            check(p["cross_b"][l], new["cross_b"][l], idx)
    check(p["dnn_hidden"][0][0], new["dnn_hidden"][0][0], (3, 2))
    check(p["dnn_hidden"][0][1], new["dnn_hidden"][0][1], (1,))
    check(p["dnn_out"][0], new["dnn_out"][0], (2, 1))
    check(p["dnn_out"][1], new["dnn_out"][1], (0,))
    for idx in [(0, 0), (5, 0), (9, 0)]:
        check(p["out_kernel"], new["out_kernel"], idx)
    check(p["out_bias"], new["out_bias"], (0,))


def test_embed_fm_train_step_gradient_matches_finite_differences():
    """oracle.embed_fm_train_step (the sharded trainer's objective) == central
    differences of its loss, for rows (one repeated), w0, w1, v."""
    rng = np.random.default_rng(14)
    nd, k, kfm = 2, 3, 2
    tables = [rng.normal(size=(v_, k)) * 0.5 for v_ in (3, 2)]
    d = nd + 2 * k
    p = {"tables": tables, "w0": np.array([0.1]), "w1": rng.normal(size=(d, 1)), "v": rng.normal(size=(d, kfm))}
    dense = rng.random((4, nd))
    ids = np.array([[0, 1], [2, 1], [0, 0], [1, 1]])
    t = np.array([1.0, 0.0, 1.0, 0.0])
    lr, l2w, l2v = 1.0, 1e-2, 3e-2
    new, _ = O.embed_fm_train_step(dense, ids, t, p, lr, l2w, l2v, nd=nd)
    eps = 1e-6

    def check(arr, new_arr, idx):
        keep = arr[idx]
        arr[idx] = keep + eps
        lp = O.embed_fm_loss(dense, ids, t, p, l2w, l2v, nd=nd)
        arr[idx] = keep - eps
        lm = O.embed_fm_loss(dense, ids, t, p, l2w, l2v, nd=nd)
        arr[idx] = keep
        assert abs((lp - lm) / (2 * eps) - (arr[idx] - new_arr[idx]) / lr) < 1e-6, idx

    for idx in [(0, 0), (0, 2), (2, 1)]:
        check(p["tables"][0], new["tables"][0], idx)
    check(p["tables"][1], new["tables"][1], (1, 2))
    check(p["w0"], new["w0"], (0,))
    for idx in [(0, 0), (5, 0)]:
        check(p["w1"], new["w1"], idx)
    for idx in [(1, 1), (6, 0)]:
        check(p["v"], new["v"], idx)


def test_pnn_bce_is_the_keras_broadcast_form():
    """O.pnn_bce == Keras' binary_crossentropy on a [B] label vector against a
    [B, 1] logit output, written out: clip to [eps, 1-eps], eps inside the
    logs, the [B, B] broadcast, mean over the last axis, then the batch mean
    (model/pnn.py:79)."""
    rng = np.random.default_rng(3)
    pre = np.concatenate([rng.random(5), [-0.3, 1.7]])  # two outside the clip range
    t = np.array([1, 0, 1, 1, 0, 0, 1], np.float64)
    eps = 1e-7
    q = np.clip(pre, eps, 1 - eps)
    want = np.array([[-(t[j] * np.log(q[i] + eps) + (1 - t[j]) * np.log(1 - q[i] + eps)) for j in range(7)]
                     for i in range(7)]).mean(axis=1)
    mean, per = O.pnn_bce(pre[:, None], t)
    np.testing.assert_allclose(per, want, rtol=1e-13)
    assert abs(mean - want.mean()) < 1e-13


def test_pnn_train_step_gradient_matches_finite_differences():
    """oracle.pnn_train_step's hand backprop (the Keras-broadcast BCE on the
    logit, the DNN, the inner products' e_i . e_j backward, embedding
    scatter-add) == central differences of the PNN loop's objective, for
    embedding rows (one repeated), every DNN layer's weights and biases; the
    outputs sit inside the clip range."""
    rng = np.random.default_rng(21)
    k = 3
    vocab = [3, 2, 4]
    tables = [rng.normal(size=(v_, k)) * 0.5 for v_ in vocab]
    F = len(vocab)
    w = F * k + F * (F - 1) // 2
    p = {"tables": tables,
         "dnn_hidden": [(rng.normal(size=(w, 5)) * 0.3, rng.normal(size=5) * 0.1),
                        (rng.normal(size=(5, 3)) * 0.3, rng.normal(size=3) * 0.1)],
         "dnn_out": (rng.normal(size=(3, 1)) * 0.1, np.array([0.5]))}
    ids = np.array([[0, 1, 3], [2, 1, 0], [0, 0, 3], [1, 1, 2]])
    t = np.array([1.0, 0.0, 1.0, 0.0])
    lr = 1.0
    new, loss = O.pnn_train_step(ids, t, p, lr)
    assert loss.shape == (4,)
    eps = 1e-6

    def check(arr, new_arr, idx):
        keep = arr[idx]
        arr[idx] = keep + eps
        lp = O.pnn_loss(ids, t, p)
        arr[idx] = keep - eps
        lm = O.pnn_loss(ids, t, p)
        arr[idx] = keep
        assert abs((lp - lm) / (2 * eps) - (arr[idx] - new_arr[idx]) / lr) < 1e-6, idx

    for c, idx in [(0, (0, 0)), (0, (2, 1)), (1, (1, 2)), (2, (3, 0)), (2, (0, 1))]:
        check(p["tables"][c], new["tables"][c], idx)
    for li in range(2):
        for idx in [(0, 0), (2, 1)]:
            check(p["dnn_hidden"][li][0], new["dnn_hidden"][li][0], idx)
        check(p["dnn_hidden"][li][1], new["dnn_hidden"][li][1], (1,))
    check(p["dnn_out"][0], new["dnn_out"][0], (2, 0))
    check(p["dnn_out"][1], new["dnn_out"][1], (0,))


def _din_small(rng, nb=2, kb=2, ko=3, T=4, B=6, att=(5, 3), dnn=(6, 4)):
    beh = [f"b{i}" for i in range(nb)]
    sparse = ["u"] + beh
    dense = ["d0", "d1"]
    vb, vo = 7, 5
    K = nb * kb
    p = {"sparse_tables": {"u": rng.normal(size=(vo, ko))},
         "seq_tables": {f: rng.normal(size=(vb, kb)) for f in beh}}
    n, pr = 4 * K, []
    for h in att:
        pr.append((rng.normal(size=(n, h)) * 0.5, rng.normal(size=h) * 0.1, rng.normal(size=(T, h)) * 0.3))
        n = h
    p["att"] = {"prelu": pr, "out": (rng.normal(size=(n, 1)), np.array([0.1]))}
    D = 2 * K + ko + len(dense)
    p["bn"] = (1.0 + 0.1 * rng.normal(size=D), 0.1 * rng.normal(size=D), np.zeros(D), np.ones(D), 1e-3)
    n, dl = D, []
    for u in dnn:
        dl.append((rng.normal(size=(n, u)) * 0.4, rng.normal(size=u) * 0.1, rng.normal(size=u) * 0.2))
        n = u
    p["dnn"] = dl
    p["out"] = (rng.normal(size=(n, 1)) * 0.5, np.array([0.05]))
    hist = rng.integers(0, vb, size=(B, T, nb))
    hist[1, 2:, 0] = 0  # padded tail
    hist[3, :, 0] = 0   # fully masked row
    inputs = {"d0": rng.random((B, 1)), "d1": rng.random((B, 1)), "u": rng.integers(0, vo, (B, 1)),
              "movie_id": rng.integers(1, vb, (B, nb))}
    for i, f in enumerate(beh):
        inputs[f] = hist[:, :, i]
    t = (rng.random(B) < 0.5).astype(np.float64)
    return inputs, t, p, dense, sparse, beh


def test_din_train_step_gradient_matches_finite_differences():
    """oracle.din_train_step's hand backprop (training-mode BatchNormalization,
    Dense + PReLU layers incl. the attention's [T, h] alphas, the masked
    softmax pool with a padded and a fully masked row, the [q, k, q-k, q*k]
    concat, two behaviour features concatenated along k, embedding
    scatter-add) == central differences of compile_fit's DIN objective."""
    rng = np.random.default_rng(7)
    inputs, t, p, dense, sparse, beh = _din_small(rng)
    lr = 1.0
    new, loss = O.din_train_step(inputs, t, p, dense, sparse, beh, lr)
    assert loss.shape == (6,)
    eps = 1e-6

    def check(get, idx, get_new):
        arr = get(p)
        keep = arr[idx]
        arr[idx] = keep + eps
        lp = O.din_loss(inputs, t, p, dense, sparse, beh)
        arr[idx] = keep - eps
        lm = O.din_loss(inputs, t, p, dense, sparse, beh)
        arr[idx] = keep
        fd = (lp - lm) / (2 * eps)
        got = (arr[idx] - get_new(new)[idx]) / lr
        assert abs(fd - got) < 1e-6 * max(1.0, abs(fd)), (idx, fd, got)

    for f in beh:
        for idx in [(0, 0), (2, 1), (4, 0), (5, 1)]:
            check(lambda q, f=f: q["seq_tables"][f], idx, lambda q, f=f: q["seq_tables"][f])
    for idx in [(1, 2), (3, 0)]:
        check(lambda q: q["sparse_tables"]["u"], idx, lambda q: q["sparse_tables"]["u"])
    for li in range(2):
        for j, idx in [(0, (1, 1)), (0, (4, 0)), (1, (2,)), (2, (1, 2)), (2, (3, 0))]:
            check(lambda q, li=li, j=j: q["att"]["prelu"][li][j], idx, lambda q, li=li, j=j: q["att"]["prelu"][li][j])
    check(lambda q: q["att"]["out"][0], (1, 0), lambda q: q["att"]["out"][0])
    check(lambda q: q["att"]["out"][1], (0,), lambda q: q["att"]["out"][1])
    for j, idx in [(0, (2,)), (0, (9,)), (1, (4,))]:
        check(lambda q, j=j: q["bn"][j], idx, lambda q, j=j: q["bn"][j])
    for li in range(2):
        for j, idx in [(0, (0, 1)), (1, (2,)), (2, (1,))]:
            check(lambda q, li=li, j=j: q["dnn"][li][j], idx, lambda q, li=li, j=j: q["dnn"][li][j])
    check(lambda q: q["out"][0], (2, 0), lambda q: q["out"][0])
    check(lambda q: q["out"][1], (0,), lambda q: q["out"][1])
    # moving statistics: momentum 0.99 toward the batch mean / biased variance
    c = O._din_train_forward(inputs, p, dense, sparse, beh, np.float64)
    np.testing.assert_allclose(new["bn"][2], 0.01 * c["bmu"], rtol=1e-12)
    np.testing.assert_allclose(new["bn"][3], 0.99 + 0.01 * c["bvar"], rtol=1e-12)


@pytest.mark.parametrize("mode", ["outer", "both"])
def test_pnn_train_step_outer_gradient_matches_finite_differences(mode):
    """The same for modes 'outer' / 'both' (the reference loop's own example,
    model/pnn.py:61): the OuterProductLayer weight W [k, P, k] and the rows
    feeding the outer products o_p = e_j^T W_p e_i, against central
    differences of the loop's objective."""
    rng = np.random.default_rng(22)
    k = 3
    vocab = [3, 2, 4]
    F = len(vocab)
    P = F * (F - 1) // 2
    tables = [rng.normal(size=(v_, k)) * 0.5 for v_ in vocab]
    w = F * k + (2 if mode == "both" else 1) * P
    p = {"tables": tables, "outer_W": rng.normal(size=(k, P, k)) * 0.4,
         "dnn_hidden": [(rng.normal(size=(w, 5)) * 0.3, rng.normal(size=5) * 0.1)],
         "dnn_out": (rng.normal(size=(5, 1)) * 0.1, np.array([0.5]))}
    ids = np.array([[0, 1, 3], [2, 1, 0], [0, 0, 3], [1, 1, 2]])
    t = np.array([1.0, 0.0, 1.0, 0.0])
    lr = 1.0
    new, _ = O.pnn_train_step(ids, t, p, lr, mode=mode)
    eps = 1e-6

    def check(arr, new_arr, idx):
        keep = arr[idx]
        arr[idx] = keep + eps
        lp = O.pnn_loss(ids, t, p, mode=mode)
        arr[idx] = keep - eps
        lm = O.pnn_loss(ids, t, p, mode=mode)
        arr[idx] = keep
        assert abs((lp - lm) / (2 * eps) - (arr[idx] - new_arr[idx]) / lr) < 1e-6, idx

    for idx in [(0, 0, 0), (2, 1, 1), (1, 2, 0), (0, 2, 2)]:
        check(p["outer_W"], new["outer_W"], idx)
    for c, idx in [(0, (0, 0)), (0, (2, 1)), (1, (1, 2)), (2, (3, 0))]:
        check(p["tables"][c], new["tables"][c], idx)
    check(p["dnn_hidden"][0][0], new["dnn_hidden"][0][0], (w - 1, 2))


@pytest.mark.parametrize("att_act,dnn_act", [("dice", "prelu"), ("prelu", "dice"), ("dice", "dice")])
def test_din_train_step_dice_gradient_matches_finite_differences(att_act, dnn_act):
    """The same with Dice (layer/interaction.py:410-425) in the attention
    (len(hidden) Dice layers on the 4k-wide concat, no Dense) and / or the DNN
    (Dense(unit, activation=Dice())): training-mode batch statistics inside
    Dice, its BatchNormalization backward, the alphas; the Dice moving
    averages move toward the batch mean / biased variance."""
    rng = np.random.default_rng(8)
    inputs, t, p, dense, sparse, beh = _din_small(rng)
    K = 4
    if att_act == "dice":
        p["att"] = {"dice": [(rng.normal(size=4 * K) * 0.3, np.zeros(4 * K), np.ones(4 * K), 1e-9) for _ in range(2)],
                    "out": (rng.normal(size=(4 * K, 1)), np.array([0.1]))}
    if dnn_act == "dice":
        p["dnn"] = [(W, b, (rng.normal(size=b.shape[0]) * 0.3, np.zeros(b.shape[0]), np.ones(b.shape[0]), 1e-9))
                    for W, b, _ in p["dnn"]]
    lr = 1.0
    kw = dict(att_act=att_act, dnn_act=dnn_act)
    new, _ = O.din_train_step(inputs, t, p, dense, sparse, beh, lr, **kw)
    eps = 1e-6

    def check(get, idx, get_new):
        arr = get(p)
        keep = arr[idx]
        arr[idx] = keep + eps
        lp = O.din_loss(inputs, t, p, dense, sparse, beh, **kw)
        arr[idx] = keep - eps
        lm = O.din_loss(inputs, t, p, dense, sparse, beh, **kw)
        arr[idx] = keep
        fd = (lp - lm) / (2 * eps)
        got = (arr[idx] - get_new(new)[idx]) / lr
        assert abs(fd - got) < 1e-5 * max(1.0, abs(fd)), (idx, fd, got)

    for f in beh:
        for idx in [(0, 0), (2, 1), (5, 1)]:
            check(lambda q, f=f: q["seq_tables"][f], idx, lambda q, f=f: q["seq_tables"][f])
    check(lambda q: q["sparse_tables"]["u"], (1, 2), lambda q: q["sparse_tables"]["u"])
    if att_act == "dice":
        for li in range(2):
            for idx in [(1,), (9,), (14,)]:
                check(lambda q, li=li: q["att"]["dice"][li][0], idx, lambda q, li=li: q["att"]["dice"][li][0])
        saved = O._din_train_forward(inputs, p, dense, sparse, beh, np.float64, **kw)["att_pre"][0]
        np.testing.assert_allclose(new["att"]["dice"][0][1], 0.01 * saved[0], rtol=1e-12)
    check(lambda q: q["att"]["out"][0], (1, 0), lambda q: q["att"]["out"][0])
    for li in range(2):
        check(lambda q, li=li: q["dnn"][li][0], (0, 1), lambda q, li=li: q["dnn"][li][0])
        check(lambda q, li=li: q["dnn"][li][1], (2,), lambda q, li=li: q["dnn"][li][1])
        if dnn_act == "dice":
            check(lambda q, li=li: q["dnn"][li][2][0], (1,), lambda q, li=li: q["dnn"][li][2][0])
    for j, idx in [(0, (2,)), (1, (4,))]:
        check(lambda q, j=j: q["bn"][j], idx, lambda q, j=j: q["bn"][j])


def test_nfm_train_step_gradient_matches_finite_differences():
    """oracle.nfm_train_step (compile_fit on NFM: training-mode BN, the
    Bi-Interaction backward de_f = dbi (S - e_f), relu DNNLayer + linear
    output + Dense(1), embedding scatter-add) == central differences."""
    rng = np.random.default_rng(31)
    k, vocab, nd = 3, [3, 2, 4], 2
    tables = [rng.normal(size=(v_, k)) * 0.7 for v_ in vocab]
    D = nd + k
    p = {"tables": tables, "bn": (1 + 0.1 * rng.normal(size=D), 0.1 * rng.normal(size=D), np.zeros(D), np.ones(D), 1e-3),
         "dnn_hidden": [(rng.normal(size=(D, 5)) * 0.5, rng.normal(size=5) * 0.1)],
         "dnn_out": (rng.normal(size=(5, 2)) * 0.5, rng.normal(size=2) * 0.1),
         "out": (rng.normal(size=(2, 1)), np.array([0.1]))}
    ids = np.array([[0, 1, 3], [2, 1, 0], [0, 0, 3], [1, 1, 2], [2, 0, 1]])
    dense = rng.random((5, nd))
    t = np.array([1.0, 0.0, 1.0, 0.0, 1.0])
    new, _ = O.nfm_train_step(dense, ids, t, p, 1.0)
    eps = 1e-6

    def check(arr, new_arr, idx):
        keep = arr[idx]
        arr[idx] = keep + eps
        lp = O.nfm_loss(dense, ids, t, p)
        arr[idx] = keep - eps
        lm = O.nfm_loss(dense, ids, t, p)
        arr[idx] = keep
        assert abs((lp - lm) / (2 * eps) - (arr[idx] - new_arr[idx])) < 1e-6, idx

    for c, idx in [(0, (0, 0)), (0, (2, 1)), (1, (1, 2)), (2, (3, 0))]:
        check(p["tables"][c], new["tables"][c], idx)
    check(p["dnn_hidden"][0][0], new["dnn_hidden"][0][0], (3, 2))
    check(p["dnn_out"][0], new["dnn_out"][0], (1, 1))
    check(p["out"][0], new["out"][0], (0, 0))
    check(p["out"][1], new["out"][1], (0,))
    for j, idx in [(0, (2,)), (1, (4,))]:
        check(p["bn"][j], new["bn"][j], idx)


def test_nfm_din_train_steps_with_dropout_match_finite_differences():
    """oracle.nfm_train_step / din_train_step with fixed dropout multipliers
    (NFM: after each hidden layer, interaction.py:44; DIN: after the DNN,
    din.py:93) == central differences of the same masked objective."""
    rng = np.random.default_rng(33)
    k, vocab, nd = 3, [3, 2, 4], 2
    D = nd + k
    p = {"tables": [rng.normal(size=(v_, k)) * 0.7 for v_ in vocab],
         "bn": (1 + 0.1 * rng.normal(size=D), 0.1 * rng.normal(size=D), np.zeros(D), np.ones(D), 1e-3),
         "dnn_hidden": [(rng.normal(size=(D, 5)) * 0.5, rng.normal(size=5) * 0.1),
                        (rng.normal(size=(5, 4)) * 0.5, rng.normal(size=4) * 0.1)],
         "dnn_out": (rng.normal(size=(4, 2)) * 0.5, rng.normal(size=2) * 0.1),
         "out": (rng.normal(size=(2, 1)), np.array([0.1]))}
    ids = np.array([[0, 1, 3], [2, 1, 0], [0, 0, 3], [1, 1, 2], [2, 0, 1]])
    dense = rng.random((5, nd))
    t = np.array([1.0, 0.0, 1.0, 0.0, 1.0])
    masks = [O.dropout_multiplier(5, w, 0.3, 11, off) for w, off in ((5, 0), (4, 28))]
    assert any((m_ == 0).any() for m_ in masks)
    new, _ = O.nfm_train_step(dense, ids, t, p, 1.0, masks=masks)
    eps = 1e-6

    def check(loss_fn, arr, new_arr, idx):
        keep = arr[idx]
        arr[idx] = keep + eps
        lp = loss_fn()
        arr[idx] = keep - eps
        lm = loss_fn()
        arr[idx] = keep
        fd = (lp - lm) / (2 * eps)
        assert abs(fd - (arr[idx] - new_arr[idx])) < 1e-6 * max(1.0, abs(fd)), (idx, fd)

    nl = lambda: O.nfm_loss(dense, ids, t, p, masks=masks)
    for c, idx in [(0, (0, 0)), (2, (3, 0))]:
        check(nl, p["tables"][c], new["tables"][c], idx)
    for li in range(2):
        check(nl, p["dnn_hidden"][li][0], new["dnn_hidden"][li][0], (1, 2))
        check(nl, p["dnn_hidden"][li][1], new["dnn_hidden"][li][1], (3,))
    check(nl, p["dnn_out"][0], new["dnn_out"][0], (1, 1))
    check(nl, p["bn"][0], new["bn"][0], (2,))

    inputs, t, p, dense_f, sparse_f, beh = _din_small(rng)
    B = len(t)
    h = np.asarray(p["dnn"][-1][0]).shape[1]
    mask = O.dropout_multiplier(B, h, 0.4, 5, 0)
    assert (mask == 0).any()
    new, _ = O.din_train_step(inputs, t, p, dense_f, sparse_f, beh, 1.0, drop_mask=mask)
    dl = lambda: O.din_loss(inputs, t, p, dense_f, sparse_f, beh, drop_mask=mask)
    check(dl, p["out"][0], new["out"][0], (1, 0))
    for li in range(len(p["dnn"])):
        check(dl, p["dnn"][li][0], new["dnn"][li][0], (0, 1))
        check(dl, p["dnn"][li][2], new["dnn"][li][2], (1,))
    f = beh[0]
    check(dl, p["seq_tables"][f], new["seq_tables"][f], (2, 1))
    check(dl, p["bn"][0], new["bn"][0], (2,))


def test_ffm_train_step_gradient_matches_finite_differences():
    """oracle.ffm_train_step (compile_fit on FFM: BCE + l2(w_reg) on w + l2(v_reg)
    on v, the field-aware interaction's G = g (T - Fm)) == central differences
    of ffm_loss, on dense rows, looked-up rows (one repeated) and w0."""
    rng = np.random.default_rng(41)
    dims, nd, k = [3, 2, 4], 2, 3
    NF, nfeat = nd + len(dims), nd + sum(dims)
    w0 = np.array([0.1])
    w = rng.normal(size=(nfeat, 1)) * 0.3
    v = rng.normal(size=(nfeat, NF, k)) * 0.3
    dense = rng.random((5, nd))
    ids = np.array([[0, 1, 3], [2, 1, 0], [0, 0, 3], [1, 1, 2], [2, 0, 1]])
    t = np.array([1.0, 0.0, 1.0, 0.0, 1.0])
    l2w, l2v = 1e-2, 2e-2
    (nw0, nw, nv), _ = O.ffm_train_step(dense, ids, t, w0, w, v, dims, 1.0, l2w, l2v)
    eps = 1e-6

    def check(arr, new_arr, idx):
        keep = arr[idx]
        arr[idx] = keep + eps
        lp = O.ffm_loss(dense, ids, t, w0, w, v, dims, l2w, l2v)
        arr[idx] = keep - eps
        lm = O.ffm_loss(dense, ids, t, w0, w, v, dims, l2w, l2v)
        arr[idx] = keep
        assert abs((lp - lm) / (2 * eps) - (arr[idx] - new_arr[idx])) < 1e-6, idx

    check(w0, nw0, (0,))
    for idx in [(0, 0), (2, 0), (nd + 3, 0), (nfeat - 1, 0)]:
        check(w, nw, idx)
    for idx in [(1, 0, 2), (nd + 0, 3, 1), (nd + 3, 1, 0), (nfeat - 1, 4, 2), (nd + 2, 0, 0)]:
        check(v, nv, idx)
