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


@pytest.mark.gpu
@pytest.mark.parametrize("B,k,hidden,vmax,id_dtype,drop", [(32, 8, [256, 128, 64], 5, np.int32, 0.2),
                                                           (32, 8, [256, 128, 64], 5, np.int32, False),
                                                           (300, 16, [24, 12], 50, np.int64, 0.2),
                                                           (301, 16, [24, 12], 50, np.int64, False),
                                                           (7, 4, [], 3, np.int32, 0.2)])
def test_deepfm_train_steps_match_oracle(gpu, B, k, hidden, vmax, id_dtype, drop):
    """DeepFM.train_step (gather, saved activations, DNNLayer's Dropout in
    training mode, rs_gemm backward, FM gradients, l2, SGD, row-sparse
    embedding scatter-add) == the oracle's hand backprop (pinned by finite
    differences) fed the same dropout multipliers, over 3 steps, with many
    repeated rows; the fused forward then runs on the trained weights.
    drop: the DNNLayer rate (the reference default 0.2) or False (off)."""
    import recommender_system_amd as rs
    from recommender_system_amd import models as M
    from tests.helpers import criteo_columns, dnn_params, dropout_masks, tables_of
    rng = np.random.default_rng(B + k)
    vocab = rng.integers(1, vmax, 26)
    m = rs.DeepFM(criteo_columns(vocab, embed_dim=k), 10, 1e-3, 2e-3, hidden, 1, "relu", embed_dim=k, seed=2)
    with torch.no_grad():
        m.embed_layer.table.mul_(10.0)  # O(1) activations: a visible update against fp32 rounding
        for l in m.dnn._layers():
            l.bias.uniform_(-0.1, 0.1)

    def params():
        hid, out = dnn_params(m.dnn)
        return {"tables": tables_of(m.embed_layer), "w0": m.fm.w0.cpu().numpy(), "w1": m.fm.w1.cpu().numpy(),
                "v": m.fm.v.cpu().numpy(), "dnn_hidden": hid, "dnn_out": out}

    p = {kk: vv for kk, vv in params().items()}
    lr = 0.5
    assert m.dnn.dropout == 0.2  # DNNLayer's default (layer/interaction.py:30)
    dr = M._dropout_rng(m)
    for step in range(3):
        dense = rng.random((B, 13)).astype(np.float32)
        ids = np.stack([rng.integers(0, v_, B) for v_ in vocab], 1).astype(id_dtype)
        t = rng.integers(0, 2, B).astype(np.float32)
        masks = dropout_masks(dr.seed, dr.offset, B, hidden, 0.2)[0] if drop else None
        loss = m.train_step((dense, ids), t, lr=lr, return_loss=True, dropout=None if drop else False)
        p, ce = O.deepfm_train_step(dense, ids, t, p, lr, 1e-3, 2e-3, masks=masks)
        got = params()
        assert_scaled_close(loss, ce, what=f"step {step} loss")
        for c in range(26):
            assert_scaled_close(got["tables"][c], p["tables"][c], what=f"step {step} table {c}")
        # w0 is ONE scalar: a sum over every sample of every step whose terms
        # (~lr/B each) cancel down to ~1e-4, so fp32 summation-order noise is
        # ~1e-5 of its value; its tolerance is the summands' scale, not its own
        assert_scaled_close(got["w0"], p["w0"], rtol=1e-4, what=f"step {step} w0")
        for name in ("w1", "v"):
            assert_scaled_close(got[name], p[name], what=f"step {step} {name}")
        for li, ((W, b), (Wr, br)) in enumerate(zip(got["dnn_hidden"], p["dnn_hidden"])):
            assert_scaled_close(W, Wr, what=f"step {step} W{li}")
            assert_scaled_close(b, br, what=f"step {step} b{li}")
        assert_scaled_close(got["dnn_out"][0], p["dnn_out"][0], what=f"step {step} W_out")
    y = m((dense, ids))
    assert_scaled_close(y, O.deepfm(None, p, inputs=(dense, ids))[0], what="forward after training")


@pytest.mark.gpu
def test_compile_fit_deepfm_on_bundled_sample(gpu):
    """compile_fit on DeepFM (model/deepFM.py's __main__ flow) over the
    reference's bundled Criteo sample: the loss falls epoch over epoch, and
    the first 5 SGD steps equal the oracle's."""
    import os

    import recommender_system_amd as rs
    from recommender_system_amd import models as M
    from recommender_system_amd.dataset import criteo_compact, features_dict
    from recommender_system_amd.train import compile_fit
    from tests.helpers import dnn_params, dropout_masks, tables_of
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "criteo_train_1w.txt.gz")
    dense, ids, label, _ = criteo_compact(path)
    cols = features_dict(path)
    m = rs.DeepFM(cols, 10, 1e-4, 1e-4, [64, 32], 1, "relu", seed=4)
    hid, out = dnn_params(m.dnn)
    p = {"tables": tables_of(m.embed_layer), "w0": m.fm.w0.cpu().numpy(), "w1": m.fm.w1.cpu().numpy(),
         "v": m.fm.v.cpu().numpy(), "dnn_hidden": hid, "dnn_out": out}
    N = 160
    dr = M._dropout_rng(m)  # fit runs DNNLayer's Dropout(0.2): the oracle gets the same draws
    seed, off = dr.seed, dr.offset
    compile_fit(m, dense[:N], ids[:N], label[:N], batch_size=32, epochs=1, sgd=0.01)
    d32 = dense[:N].astype(np.float32)
    for r0 in range(0, N, 32):
        masks, off = dropout_masks(seed, off, 32, [64, 32], 0.2)
        p, _ = O.deepfm_train_step(d32[r0:r0 + 32], ids[r0:r0 + 32], label[r0:r0 + 32], p, 0.01, 1e-4, 1e-4,
                                   masks=masks)
    assert_scaled_close(m.fm.v, p["v"], what="DeepFM compile_fit v")
    for c in (0, 7, 25):
        assert_scaled_close(m.embed_layer.field_table(c), p["tables"][c], what=f"DeepFM compile_fit table {c}")
    m2 = rs.DeepFM(cols, 10, 1e-4, 1e-4, [64, 32], 1, "relu", seed=4)
    hist = compile_fit(m2, dense[:960], ids[:960], label[:960], batch_size=32, epochs=4, sgd=0.05)
    assert hist[-1] < hist[0]


def _dcn_params(m):
    from tests.helpers import dnn_params, tables_of
    hid, out = dnn_params(m.dense_layer)
    return {"tables": tables_of(m.embed_layer),
            "cross_w": [w.detach().cpu().numpy() for w in m.cross_layer.cross_weight],
            "cross_b": [b.detach().cpu().numpy() for b in m.cross_layer.cross_bias],
            "dnn_hidden": hid, "dnn_out": out,
            "out_kernel": m.output_layer.kernel.detach().cpu().numpy(),
            "out_bias": m.output_layer.bias.detach().cpu().numpy()}


@pytest.mark.gpu
@pytest.mark.parametrize("B,k,hidden,od,L,vmax,id_dtype,drop", [(32, 8, [64, 32], 4, 3, 5, np.int32, 0.2),
                                                                (33, 8, [64, 32], 4, 3, 5, np.int32, False),
                                                                (300, 16, [24], 1, 2, 50, np.int64, 0.2),
                                                                (7, 4, [], 2, 0, 3, np.int32, 0.2)])
def test_dcn_train_steps_match_oracle(gpu, B, k, hidden, od, L, vmax, id_dtype, drop):
    """DCN.train_step (rs_cross_train_fwd / _bwd, DNNLayer's Dropout in
    training mode, output Dense and DNN through rs_gemm / rs_col_sum,
    CrossLayer l2, SGD, row-sparse embedding update) == the oracle's hand
    backprop (pinned by finite differences) fed the same dropout multipliers
    over 3 steps; the fused forward then runs on the trained weights."""
    import recommender_system_amd as rs
    from recommender_system_amd import models as M
    from tests.helpers import criteo_columns, dropout_masks
    rng = np.random.default_rng(B + k + L)
    vocab = rng.integers(1, vmax, 26)
    m = rs.DCN(criteo_columns(vocab, embed_dim=k), hidden, od, "relu", layer_num=L, reg_w=1e-3, reg_b=2e-3,
               embed_dim=k, seed=3)
    with torch.no_grad():
        m.embed_layer.table.mul_(10.0)
        for l in m.dense_layer._layers():
            l.bias.uniform_(-0.1, 0.1)
        m.output_layer.bias.uniform_(-0.1, 0.1)
    p = _dcn_params(m)
    lr = 0.5
    dr = M._dropout_rng(m)
    for step in range(3):
        dense = rng.random((B, 13)).astype(np.float32)
        ids = np.stack([rng.integers(0, v_, B) for v_ in vocab], 1).astype(id_dtype)
        t = rng.integers(0, 2, B).astype(np.float32)
        masks = dropout_masks(dr.seed, dr.offset, B, hidden, 0.2)[0] if drop else None
        loss = m.train_step((dense, ids), t, lr=lr, return_loss=True, dropout=None if drop else False)
        p, ce = O.dcn_train_step(dense, ids, t, p, lr, 1e-3, 2e-3, masks=masks)
        got = _dcn_params(m)
        assert_scaled_close(loss, ce, what=f"step {step} loss")
        for c in range(26):
            assert_scaled_close(got["tables"][c], p["tables"][c], what=f"step {step} table {c}")
        for l in range(L):
            assert_scaled_close(got["cross_w"][l], p["cross_w"][l], what=f"step {step} w{l}")
            assert_scaled_close(got["cross_b"][l], p["cross_b"][l], what=f"step {step} b{l}")
        for li, ((W, b), (Wr, br)) in enumerate(zip(got["dnn_hidden"], p["dnn_hidden"])):
            assert_scaled_close(W, Wr, what=f"step {step} W{li}")
            assert_scaled_close(b, br, what=f"step {step} b{li}")
        assert_scaled_close(got["dnn_out"][0], p["dnn_out"][0], what=f"step {step} dnn W_out")
        assert_scaled_close(got["out_kernel"], p["out_kernel"], what=f"step {step} out kernel")
        assert_scaled_close(got["out_bias"], p["out_bias"], what=f"step {step} out bias")
    y = m((dense, ids))
    assert_scaled_close(y, O.dcn(None, dict(p, act="relu"), inputs=(dense, ids))[0], what="forward after training")


@pytest.mark.gpu
def test_compile_fit_dcn_on_bundled_sample(gpu):
    """compile_fit on DCN (model/dcn.py's __main__ flow, layer_num 3) over the
    reference's bundled Criteo sample: the first 5 SGD steps equal the
    oracle's, and the loss falls epoch over epoch."""
    import os

    import recommender_system_amd as rs
    from recommender_system_amd import models as M
    from recommender_system_amd.dataset import criteo_compact, features_dict
    from recommender_system_amd.train import compile_fit
    from tests.helpers import dropout_masks
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "criteo_train_1w.txt.gz")
    dense, ids, label, _ = criteo_compact(path)
    cols = features_dict(path)
    m = rs.DCN(cols, [64, 32], 1, "relu", 3, seed=5)
    p = _dcn_params(m)
    N = 160
    dr = M._dropout_rng(m)  # fit runs DNNLayer's Dropout(0.2): the oracle gets the same draws
    seed, off = dr.seed, dr.offset
    compile_fit(m, dense[:N], ids[:N], label[:N], batch_size=32, epochs=1, sgd=0.01)
    d32 = dense[:N].astype(np.float32)
    for r0 in range(0, N, 32):
        masks, off = dropout_masks(seed, off, 32, [64, 32], 0.2)
        p, _ = O.dcn_train_step(d32[r0:r0 + 32], ids[r0:r0 + 32], label[r0:r0 + 32], p, 0.01, 1e-4, 1e-4,
                                masks=masks)
    got = _dcn_params(m)
    for l in range(3):
        assert_scaled_close(got["cross_w"][l], p["cross_w"][l], what=f"DCN compile_fit w{l}")
    for c in (0, 7, 25):
        assert_scaled_close(got["tables"][c], p["tables"][c], what=f"DCN compile_fit table {c}")
    m2 = rs.DCN(cols, [64, 32], 1, "relu", 3, seed=5)
    hist = compile_fit(m2, dense[:960], ids[:960], label[:960], batch_size=32, epochs=4, sgd=0.05)
    assert hist[-1] < hist[0]


@pytest.mark.gpu
@pytest.mark.parametrize("ta,tb", [(0, 0), (1, 0), (0, 1), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(4096, 256, 429), (429, 256, 4096), (37, 1, 70), (64, 65, 16), (3, 5, 0)])
def test_rs_gemm_mfma_matches_torch(gpu, ta, tb, M, N, K):
    """rs_gemm (v_mfma_f32_32x32x2_f32 tiles, split-K through the workspace
    when K is long) == a torch fp64 GEMM of the same fp32 operands, with
    alpha / beta / the ReLU-mask epilogue; bitwise run to run."""
    from recommender_system_amd import _lib
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N * 3 + K + ta * 2 + tb)
    A = torch.randn(*((K, M) if ta else (M, K)), generator=g).to(gpu)
    B = torch.randn(*((N, K) if tb else (K, N)), generator=g).to(gpu)
    C0 = torch.randn(M, N, generator=g).to(gpu)
    mask = (torch.rand(M, N, generator=g) > 0.3).float().to(gpu)
    ws = torch.empty(max(int(_lib.lib().rs_gemm_workspace_size(M, N, K)), 1), dtype=torch.uint8, device=gpu)
    st = _lib.stream()
    outs = []
    for _ in range(2):
        C = C0.clone()
        _lib.call("rs_gemm", ta, tb, M, N, K, 0.5, A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), 2.0,
                  C.data_ptr(), N, mask.data_ptr(), N, ws.data_ptr(), ws.numel(), st)
        outs.append(C.cpu())
    opA = (A.T if ta else A).double().cpu()
    opB = (B.T if tb else B).double().cpu()
    ref = (0.5 * (opA @ opB) + 2.0 * C0.double().cpu()) * mask.double().cpu()
    scale = float(opA.abs().sum(1).max() * opB.abs().max()) if K else 1.0
    assert float((outs[0].double() - ref).abs().max()) <= 2e-6 * max(scale, 1.0)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.gpu
def test_dropout_counter_under_graph_replay(gpu):
    """The dropout offset lives in device memory (rs_dropout_at /
    rs_dropout_advance): a captured draw + advance replays a FRESH mask on
    every replay, each equal to oracle.dropout_multiplier at the counter's
    value, and a redraw at the same relative offset inside the step repeats
    the step's mask (the backward's regeneration)."""
    from recommender_system_amd import models as M
    rng = M._Dropout(7)
    rows, cols, rate = 64, 30, 0.25
    x = torch.empty(rows, cols, device="cuda")
    y = torch.empty(rows, cols, device="cuda")
    st = lambda: torch.cuda.current_stream().cuda_stream

    def step():
        x.fill_(1.0)
        y.fill_(1.0)
        off = rng.draw(x, rate, st())
        rng.redraw(y, rate, off, st())
        rng.end_step(st())

    step()  # eager, offset 0
    torch.cuda.synchronize()
    np.testing.assert_array_equal(x.cpu().numpy(), O.dropout_multiplier(rows, cols, rate, rng.seed, 0, np.float32))
    n = (rows * cols + 3) // 4 * 4
    assert rng.offset == n
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    assert rng.offset == n  # capture ran nothing
    seen = []
    for r in range(3):
        g.replay()
        torch.cuda.synchronize()
        ref = O.dropout_multiplier(rows, cols, rate, rng.seed, n * (r + 1), np.float32)
        np.testing.assert_array_equal(x.cpu().numpy(), ref)
        assert torch.equal(x, y)
        seen.append(x.clone())
    assert not torch.equal(seen[0], seen[1]) and not torch.equal(seen[1], seen[2])
    assert rng.offset == 4 * n


@pytest.mark.gpu
@pytest.mark.parametrize("rows,cols,ld,rate,offset", [(4096, 256, 256, 0.2, 0), (33, 7, 9, 0.5, 1236),
                                                      (1, 3, 3, 0.2, 4), (300, 24, 24, 0.0, 8)])
def test_rs_dropout_matches_oracle_generator(gpu, rows, cols, ld, rate, offset):
    """rs_dropout == oracle.dropout_multiplier bit for bit (Philox4x32-10
    draws, keep = u >= rate, scale 1/(1-rate)) on a strided tensor, padding
    columns untouched; applying it again with the same (seed, offset) is the
    backward (keep^2 = keep, one more scale)."""
    from recommender_system_amd import _lib
    g = torch.Generator(device="cpu").manual_seed(rows + cols)
    x0 = torch.randn(rows, ld, generator=g)
    x = x0.clone().to(gpu)
    seed = 0x1234_5678_9ABC_DEF0
    _lib.call("rs_dropout", x.data_ptr(), ld, rows, cols, rate, seed, offset, _lib.stream())
    m = O.dropout_multiplier(rows, cols, rate, seed, offset, np.float32)
    ref = x0.numpy().copy()
    ref[:, :cols] = ref[:, :cols] * m
    np.testing.assert_array_equal(x.cpu().numpy(), ref)
    if rate > 0 and rows * cols > 1000:
        assert abs(float((m == 0).mean()) - rate) < 0.01


@pytest.mark.gpu
@pytest.mark.parametrize("B,k,hidden,mode", [(32, 8, [64, 32], "inner"), (300, 16, [256, 128, 64], "inner"),
                                             (64, 8, [64, 32], "outer"), (300, 16, [256, 128, 64], "both")])
def test_pnn_train_steps_match_oracle(gpu, B, k, hidden, mode):
    """PNN.train_step (the reference's GradientTape loop, its Keras-broadcast
    BCE on the logit, DNN backward, inner- and outer-product backward
    (rs_outer_product_bwd / _w_grad), SGD of the DNN and of W, row-sparse
    embedding SGD) == oracle.pnn_train_step (pinned by finite differences)
    over 3 steps with repeated rows, modes 'inner' / 'outer' / 'both'; the
    forward then runs on the trained weights."""
    import recommender_system_amd as rs
    from tests.helpers import criteo_columns, dnn_params, tables_of
    rng = np.random.default_rng(B + k + (0 if mode == "inner" else len(mode)))
    vocab = rng.integers(1, 300, 26)
    m = rs.PNN(criteo_columns(vocab, embed_dim=k), mode, hidden, 1, "relu", embed_dim=k, seed=4)
    outer = mode in ("outer", "both")
    with torch.no_grad():
        m.embed_layer.table.mul_(8.0)  # O(1) products: visible row updates
        m.dnn_layer.output_layer.bias.fill_(0.5)  # logits inside the clip range
        m.dnn_layer.output_layer.kernel.mul_(0.1)
        if outer:
            m.outer_product_layer.W.mul_(4.0)

    def params():
        hid, out = dnn_params(m.dnn_layer)
        q = {"tables": tables_of(m.embed_layer), "dnn_hidden": hid, "dnn_out": out}
        if outer:
            q["outer_W"] = m.outer_product_layer.W.cpu().numpy().astype(np.float64)
        return q

    p = params()
    lr = 0.5
    for step in range(3):
        dense = rng.random((B, 13)).astype(np.float32)
        ids = np.stack([rng.integers(0, v_, B) for v_ in vocab], 1).astype(np.int32)
        ids[:5, 4] = 0  # repeated rows
        t = rng.integers(0, 2, B).astype(np.float32)
        loss = m.train_step((dense, ids), t, lr=lr, return_loss=True)
        p, ce = O.pnn_train_step(ids, t, p, lr, mode=mode)
        got = params()
        assert_scaled_close(loss, ce, what=f"step {step} loss")
        for c in range(26):
            assert_scaled_close(got["tables"][c], p["tables"][c], what=f"step {step} table {c}")
        for li, ((W, b), (Wr, br)) in enumerate(zip(got["dnn_hidden"], p["dnn_hidden"])):
            assert_scaled_close(W, Wr, what=f"step {step} W{li}")
            assert_scaled_close(b, br, what=f"step {step} b{li}")
        assert_scaled_close(got["dnn_out"][0], p["dnn_out"][0], what=f"step {step} W_out")
        assert_scaled_close(got["dnn_out"][1], p["dnn_out"][1], what=f"step {step} b_out")
        if outer:
            assert_scaled_close(got["outer_W"], p["outer_W"], what=f"step {step} outer W")
    y = m((dense, ids))
    assert_scaled_close(y, O.pnn(None, {**p, "act": "relu"}, mode=mode, inputs=(dense, ids))[0],
                        what="forward after training")


@pytest.mark.gpu
@pytest.mark.parametrize("k,B", [(1, 3000), (8, 3000), (16, 700), (100, 3000), (200, 1500)])
def test_embedding_sgd_hot_rows(gpu, k, B):
    """rs_embedding_sgd with rows repeated thousands of times (segments cut
    into chunk pieces and recombined, emb_piece_kernel / emb_cross_kernel),
    field offsets, a strided grad: == numpy's scatter-add in fp64 at fp32
    tolerance, and bitwise reproducible run to run."""
    from recommender_system_amd import _lib
    from recommender_system_amd._lib import call, ptr
    rng = np.random.default_rng(k + B)
    vocab = np.array([50, 9], dtype=np.int64)
    offs = np.array([0, 50], dtype=np.int64)
    F = 2
    ids = np.stack([rng.integers(0, 50, B), rng.integers(0, 9, B)], 1).astype(np.int32)
    ids[rng.random(B) < 0.6, 0] = 7  # one row ~0.6 B times
    ids[: B // 3, 1] = 4
    table0 = rng.standard_normal((59, k)).astype(np.float32)
    ldg = F * k + 3
    grad = rng.standard_normal((B, ldg)).astype(np.float32)
    lr = 0.05
    ref = table0.astype(np.float64)
    for c in range(F):
        np.add.at(ref, offs[c] + ids[:, c], -lr * grad[:, c * k:(c + 1) * k].astype(np.float64))
    dev = torch.device("cuda")
    ids_d, g_d = torch.as_tensor(ids, device=dev), torch.as_tensor(grad, device=dev)
    offs_d, voc_d = torch.as_tensor(offs, device=dev), torch.as_tensor(vocab, device=dev)
    ws = torch.empty(_lib.lib().rs_embedding_sgd_workspace_size(B * F), dtype=torch.uint8, device=dev)
    outs = []
    for _ in range(2):
        t = torch.as_tensor(table0, device=dev).clone()
        call("rs_embedding_sgd", ptr(t), 59, k, ptr(ids_d), _lib.id_kind(ids_d), ids_d.stride(0), ptr(offs_d),
             ptr(voc_d), F, B, ptr(g_d), ldg, lr, ptr(ws), None, _lib.stream())
        outs.append(t.cpu().numpy())
    assert np.array_equal(outs[0], outs[1])
    delta_ref = ref - table0
    err = np.abs((outs[0] - table0) - delta_ref)
    scale = np.maximum(np.abs(delta_ref), np.sqrt(np.mean(delta_ref ** 2)))
    assert (err <= 1e-4 * scale + 4 * np.finfo(np.float32).eps * np.abs(table0)).all(), float((err / scale).max())


@pytest.mark.gpu
@pytest.mark.parametrize("M,N", [(1, 1), (255, 63), (256, 64), (257, 65), (5000, 300), (204800, 40)])
def test_col_sum_split_matches_numpy(gpu, M, N):
    """rs_col_sum_split (256-row slices in a workspace, then the slices in
    order; one-wave-per-column finish for many slices) == the fp64 column sums,
    on a strided A, bitwise reproducible run to run."""
    from recommender_system_amd import _lib
    rng = np.random.default_rng(M + N)
    A = torch.as_tensor(rng.standard_normal((M, N + 3)).astype(np.float32), device=gpu)
    ws = torch.empty(max(int(_lib.lib().rs_col_sum_workspace_size(M, N)), 1), dtype=torch.uint8, device=gpu)
    outs = []
    for _ in range(2):
        out = torch.empty(N, device=gpu)
        _lib.call("rs_col_sum_split", A.data_ptr(), A.stride(0), M, N, out.data_ptr(), ws.data_ptr(), ws.numel(),
                  _lib.stream())
        outs.append(out.cpu().numpy())
    assert np.array_equal(outs[0], outs[1])
    ref = A.cpu().numpy().astype(np.float64)[:, :N].sum(0)
    scale = np.sqrt(M) * 4 + 1
    assert np.abs(outs[0] - ref).max() <= 1e-6 * scale, float(np.abs(outs[0] - ref).max())


@pytest.mark.gpu
def test_sgd_update_multi_matches_single(gpu):
    """rs_sgd_update_multi over 40 tensors (two launches of <= 32; sizes 0, 1,
    ragged, multi-block; the single-tensor path past 2^20 blocks is not run) == one
    rs_sgd_update per tensor, bitwise (same expression per element)."""
    from recommender_system_amd import _lib
    rng = np.random.default_rng(5)
    sizes = [0, 1, 3, 1023, 1024, 1025, 70000] + [int(s) for s in rng.integers(1, 5000, 33)]
    ws = [torch.as_tensor(rng.standard_normal(max(n, 1)).astype(np.float32), device=gpu) for n in sizes]
    gs = [torch.as_tensor(rng.standard_normal(max(n, 1)).astype(np.float32), device=gpu) for n in sizes]
    l2 = [float(v) for v in rng.uniform(0, 0.1, len(sizes))]
    ref = [w.clone() for w in ws]
    st = _lib.stream()
    for w, g, n, c in zip(ref, gs, sizes, l2):
        _lib.call("rs_sgd_update", w.data_ptr(), g.data_ptr(), n, 0.05, c, st)
    _lib.sgd_update_multi([(w, g, n, c) for w, g, n, c in zip(ws, gs, sizes, l2)], 0.05, st)
    for j, (a, b) in enumerate(zip(ws, ref)):
        assert torch.equal(a, b), j


@pytest.mark.gpu
@pytest.mark.parametrize("M,N", [(1, 5), (300, 16), (20000, 64)])
def test_dice_train_fwd_bwd_match_oracle(gpu, M, N):
    """rs_dice_train_fwd / _bwd (Dice under fit: batch statistics, the
    batch-norm backward, dalpha, moving averages) == the oracle's
    _dice_train / _dice_train_bwd in fp64."""
    from recommender_system_amd import _lib
    rng = np.random.default_rng(M * 7 + N)
    x = rng.standard_normal((M, N)) * 1.5 + 0.3
    alpha = rng.uniform(-0.5, 0.5, N)
    dy = rng.standard_normal((M, N))
    mm, mv = rng.uniform(-0.1, 0.1, N), rng.uniform(0.5, 1.5, N)
    eps = 1e-9
    t = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=gpu).contiguous()
    xd, ad, dyd, mmd, mvd = t(x), t(alpha), t(dy), t(mm), t(mv)
    mean, var, y = torch.empty(N, device=gpu), torch.empty(N, device=gpu), torch.empty(M, N, device=gpu)
    dx, dal = torch.empty(M, N, device=gpu), torch.empty(N, device=gpu)
    ws = torch.empty(int(_lib.lib().rs_dice_train_workspace_size(M, N)), dtype=torch.uint8, device=gpu)
    _lib.call("rs_dice_train_fwd", xd.data_ptr(), M, N, ad.data_ptr(), eps, 0.99, mmd.data_ptr(), mvd.data_ptr(),
              mean.data_ptr(), var.data_ptr(), y.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream())
    _lib.call("rs_dice_train_bwd", xd.data_ptr(), M, N, ad.data_ptr(), mean.data_ptr(), var.data_ptr(), eps,
              dyd.data_ptr(), dx.data_ptr(), dal.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream())
    x32 = x.astype(np.float32).astype(np.float64)
    yr, saved = O._dice_train(x32, alpha.astype(np.float32), eps, np.float64)
    dxr, dalr = O._dice_train_bwd(dy.astype(np.float32).astype(np.float64), x32, alpha.astype(np.float32), eps, saved)
    assert_scaled_close(y, yr, what="dice y")
    assert_scaled_close(mean, saved[0], what="batch mean")
    assert_scaled_close(var, saved[1], what="batch var")
    if M > 1:  # one row: var 0, xhat 0 — dx is the direct term alone
        assert_scaled_close(dx, dxr, rtol=1e-4, what="dice dx")
    assert_scaled_close(dal, dalr, rtol=1e-4, what="dice dalpha")
    assert_scaled_close(mmd, 0.99 * mm.astype(np.float32) + 0.01 * saved[0], what="moving mean")
    assert_scaled_close(mvd, 0.99 * mv.astype(np.float32) + 0.01 * saved[1], what="moving var")


@pytest.mark.gpu
@pytest.mark.parametrize("B,F,k", [(1, 2, 4), (17, 3, 8), (100, 26, 16), (33, 5, 5)])
def test_outer_product_bwd_matches_oracle(gpu, B, F, k):
    """rs_outer_product_bwd (adds sum_p g_p e_j W_p / e_i W_p^T into demb) and
    rs_outer_product_w_grad (dW) == the oracle's OuterProductLayer backward,
    partial 16-sample tiles and k not a multiple of 4 included."""
    from recommender_system_amd import _lib
    rng = np.random.default_rng(B + F + k)
    P = F * (F - 1) // 2
    e = rng.standard_normal((B, F, k))
    W = rng.standard_normal((k, P, k)) * 0.3
    g = rng.standard_normal((B, P))
    base = rng.standard_normal((B, F * k))
    t = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=gpu).contiguous()
    ed, Wd, gd = t(e.reshape(B, F * k)), t(W), t(g)
    demb = t(base)
    dW = torch.empty(k, P, k, device=gpu)
    _lib.call("rs_outer_product_bwd", ed.data_ptr(), F * k, gd.data_ptr(), P, Wd.data_ptr(), F, k, B,
              demb.data_ptr(), F * k, _lib.stream())
    _lib.call("rs_outer_product_w_grad", ed.data_ptr(), F * k, gd.data_ptr(), P, F, k, B, dW.data_ptr(),
              _lib.stream())
    e32, W32, g32 = (a.astype(np.float32).astype(np.float64) for a in (e, W, g))
    row, col = O.pair_indices(F)
    de = base.astype(np.float32).astype(np.float64).reshape(B, F, k).copy()
    dWr = np.zeros_like(W32)
    for p_, (i, j) in enumerate(zip(row, col)):
        Wp = W32[:, p_, :]
        de[:, i, :] += g32[:, p_:p_ + 1] * (e32[:, j, :] @ Wp)
        de[:, j, :] += g32[:, p_:p_ + 1] * (e32[:, i, :] @ Wp.T)
        dWr[:, p_, :] = (g32[:, p_:p_ + 1] * e32[:, j, :]).T @ e32[:, i, :]
    assert_scaled_close(demb, de.reshape(B, F * k), what="demb")
    assert_scaled_close(dW, dWr, what="dW")


@pytest.mark.gpu
@pytest.mark.parametrize("B,k,hidden,rate", [(64, 8, [32, 16], 0.0), (300, 16, [256, 128, 64], 0.0),
                                             (64, 8, [32, 16], 0.3), (300, 16, [256, 128, 64], 0.3)])
def test_nfm_train_steps_match_oracle(gpu, B, k, hidden, rate):
    """NFM.train_step (compile_fit on NFM: training-mode BatchNormalization,
    the DNNLayer + output Dense backward, the Bi-Interaction backward,
    row-sparse embedding SGD) == oracle.nfm_train_step (pinned by finite
    differences) over 3 steps with repeated rows; the inference forward then
    runs on the trained weights and the moved BN averages.  rate > 0:
    NFM(dropout=rate) — DNNLayer's Dropout after each hidden layer in
    training mode, the oracle fed the same multipliers (rs_dropout's
    generator, restated by oracle.dropout_multiplier)."""
    import recommender_system_amd as rs
    from recommender_system_amd import models as M
    from tests.helpers import criteo_columns, dnn_params, dropout_masks, tables_of
    rng = np.random.default_rng(B + k + 5)
    vocab = rng.integers(1, 200, 26)
    m = rs.NFM(criteo_columns(vocab, embed_dim=k), hidden, 1, dropout=rate, embed_dim=k, seed=6)
    with torch.no_grad():
        m.emb_layers.table.mul_(4.0)

    def params():
        hid, dout = dnn_params(m.dnn_layers)
        bn = m.bn_layer
        c = lambda t: t.detach().cpu().numpy().astype(np.float64)
        return {"tables": tables_of(m.emb_layers), "dnn_hidden": hid, "dnn_out": dout,
                "out": (c(m.output_layer.kernel), c(m.output_layer.bias)),
                "bn": (c(bn.gamma), c(bn.beta), c(bn.moving_mean), c(bn.moving_variance), bn.epsilon)}

    p = params()
    lr = 0.2
    for step in range(3):
        dense = rng.random((B, 13)).astype(np.float32)
        ids = np.stack([rng.integers(0, v_, B) for v_ in vocab], 1).astype(np.int32)
        ids[:7, 3] = 0  # repeated rows
        t = rng.integers(0, 2, B).astype(np.float32)
        masks = None
        if rate:
            dr = M._dropout_rng(m)
            masks = dropout_masks(dr.seed, dr.offset, B, hidden, rate)[0]
        loss = m.train_step((dense, ids), t, lr=lr, return_loss=True)
        p, ce = O.nfm_train_step(dense, ids, t, p, lr, masks=masks)
        got = params()
        assert_scaled_close(loss, ce, what=f"step {step} loss")
        for c_ in range(26):
            assert_scaled_close(got["tables"][c_], p["tables"][c_], what=f"step {step} table {c_}")
        for li, ((W, b), (Wr, br)) in enumerate(zip(got["dnn_hidden"], p["dnn_hidden"])):
            assert_scaled_close(W, Wr, what=f"step {step} W{li}")
            assert_scaled_close(b, br, what=f"step {step} b{li}")
        for name in ("dnn_out", "out"):
            assert_scaled_close(got[name][0], p[name][0], what=f"step {step} {name} W")
            assert_scaled_close(got[name][1], p[name][1], what=f"step {step} {name} b")
        for j, nm in enumerate(("gamma", "beta", "moving_mean", "moving_variance")):
            assert_scaled_close(got["bn"][j], p["bn"][j], what=f"step {step} bn {nm}")
    pin = {"tables": p["tables"], "bn_mean": p["bn"][2], "bn_var": p["bn"][3], "bn_gamma": p["bn"][0],
           "bn_beta": p["bn"][1], "dnn_hidden": p["dnn_hidden"], "dnn_out": p["dnn_out"], "out_kernel": p["out"][0],
           "out_bias": p["out"][1]}
    assert_scaled_close(m((dense, ids)), O.nfm(None, pin, inputs=(dense, ids))[0], what="forward after training")


@pytest.mark.gpu
@pytest.mark.parametrize("B,k,vmax", [(64, 4, 9), (300, 8, 40)])
def test_ffm_train_steps_match_oracle(gpu, B, k, vmax):
    """FFM.train_step (compile_fit on FFM: BCE + l2 on every row of w and v,
    the per-sample shared gradient row G = g (T - Fm) scattered into the
    looked-up rows, dense rows through rs_gemm) == oracle.ffm_train_step
    (pinned by finite differences; one-hot formulation) over 3 steps with
    repeated rows; the forward then runs on the trained weights."""
    import recommender_system_amd as rs
    from tests.helpers import criteo_columns
    rng = np.random.default_rng(B + k)
    vocab = rng.integers(1, vmax, 26)
    m = rs.FFM(criteo_columns(vocab), k, w_reg=1e-3, v_reg=2e-3, seed=7)
    L = m.ffm
    c = lambda t: t.detach().cpu().numpy().astype(np.float64)
    w0, w, v = c(L.w0), c(L.w), c(L.v)
    lr = 0.5
    for step in range(3):
        dense = rng.random((B, 13)).astype(np.float32)
        ids = np.stack([rng.integers(0, v_, B) for v_ in vocab], 1).astype(np.int32)
        ids[:9, 2] = 0  # repeated rows
        t = rng.integers(0, 2, B).astype(np.float32)
        loss = m.train_step((dense, ids), t, lr=lr, return_loss=True)
        (w0, w, v), ce = O.ffm_train_step(dense, ids, t, w0, w, v, list(vocab), lr, 1e-3, 2e-3)
        assert_scaled_close(loss, ce, what=f"step {step} loss")
        assert_scaled_close(L.w0, w0, rtol=1e-4, what=f"step {step} w0")
        assert_scaled_close(L.w, w, what=f"step {step} w")
        assert_scaled_close(L.v, v, what=f"step {step} v")
    y = m((dense, ids))
    assert_scaled_close(y, O.sigmoid(O.ffm_layer(dense, ids, list(vocab), w0, w, v)), what="forward after training")


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["nfm", "ffm", "deepfm"])
def test_compile_fit_other_models_on_bundled_sample(gpu, which):
    """compile_fit on the reference's bundled Criteo sample for the models its
    own demos train that way (model/nfm.py:47, model/ffm.py:36,
    model/deepFM.py:47): the mean training loss falls over 3 epochs."""
    import os

    import recommender_system_amd as rs
    from recommender_system_amd.dataset import criteo_compact, features_dict
    from recommender_system_amd.train import compile_fit
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "criteo_train_1w.txt.gz")
    dense, ids, label, _ = criteo_compact(path)
    cols = features_dict(path)
    N = 640
    if which == "nfm":
        m = rs.NFM(cols, [64, 32], 1, seed=2)
    elif which == "ffm":
        m = rs.FFM(cols, 4, seed=2)
    else:
        m = rs.DeepFM(cols, 8, 1e-4, 1e-4, [64, 32], 1, "relu", seed=2)
    # FFM at the reference's own SGD(0.01) (compile_fit's default): its 39
    # field-aware sums make larger steps diverge
    hist = compile_fit(m, dense[:N], ids[:N], label[:N], batch_size=32, epochs=3, sgd=0.01 if which == "ffm" else 0.05)
    assert np.isfinite(hist).all() and hist[-1] < hist[0], hist


@pytest.mark.gpu
def test_compile_fit_din_dict_inputs(gpu):
    """compile_fit on DIN with the reference's input dict (model/din.py:106):
    batches slice every value along its first axis; the loss falls."""
    from recommender_system_amd import DIN
    from recommender_system_amd.train import compile_fit
    from tests.test_din import din_columns, din_inputs
    rng = np.random.default_rng(3)
    cols, behaviour = din_columns(1, 8, item_vocab=50, cate_vocab=9, user_vocab=17)
    inputs = din_inputs(rng, cols, behaviour, 256, 12)
    labels = rng.integers(0, 2, 256).astype(np.float32)
    m = DIN(cols, behaviour, att_hidden_units=(16, 8), dnn_hidden_units=(32, 16), seed=4)
    hist = compile_fit(m, inputs, None, labels, batch_size=32, epochs=4, sgd=0.05)
    assert np.isfinite(hist).all() and hist[-1] < hist[0], hist


@pytest.mark.gpu
def test_training_steps_single_sample_batches(gpu):
    """Batch-of-one steps (BatchNormalization's variance 0, one lookup per
    row, every reduction over a single row) for NFM, FFM, PNN 'both' and DIN
    == their oracles."""
    import recommender_system_amd as rs
    from tests.helpers import criteo_columns, dnn_params, tables_of
    from tests.test_din import din_columns, din_inputs, _din_train_params, _flat_params
    rng = np.random.default_rng(1)
    vocab = rng.integers(2, 9, 26)
    dense = rng.random((1, 13)).astype(np.float32)
    ids = np.stack([rng.integers(0, v_, 1) for v_ in vocab], 1).astype(np.int32)
    t = np.array([1.0], np.float32)
    # NFM
    m = rs.NFM(criteo_columns(vocab, embed_dim=4), [8], 1, embed_dim=4, seed=2)
    c = lambda x: x.detach().cpu().numpy().astype(np.float64)
    hid, dout = dnn_params(m.dnn_layers)
    p = {"tables": tables_of(m.emb_layers), "dnn_hidden": hid, "dnn_out": dout,
         "out": (c(m.output_layer.kernel), c(m.output_layer.bias)),
         "bn": (c(m.bn_layer.gamma), c(m.bn_layer.beta), c(m.bn_layer.moving_mean), c(m.bn_layer.moving_variance),
                m.bn_layer.epsilon)}
    loss = m.train_step((dense, ids), t, lr=0.3, return_loss=True)
    p, ce = O.nfm_train_step(dense, ids, t, p, 0.3)
    assert_scaled_close(loss, ce, what="NFM B=1 loss")
    assert_scaled_close(m.output_layer.kernel, p["out"][0], what="NFM B=1 out W")
    for c_ in range(26):
        assert_scaled_close(m.emb_layers.field_table(c_), p["tables"][c_], what=f"NFM B=1 table {c_}")
    # FFM
    f = rs.FFM(criteo_columns(vocab), 4, seed=3)
    w0, w, v = c(f.ffm.w0), c(f.ffm.w), c(f.ffm.v)
    loss = f.train_step((dense, ids), t, lr=0.3, return_loss=True)
    (w0, w, v), ce = O.ffm_train_step(dense, ids, t, w0, w, v, list(vocab), 0.3, 1e-4, 1e-4)
    assert_scaled_close(loss, ce, what="FFM B=1 loss")
    assert_scaled_close(f.ffm.v, v, what="FFM B=1 v")
    assert_scaled_close(f.ffm.w, w, what="FFM B=1 w")
    # PNN 'both'
    q = rs.PNN(criteo_columns(vocab, embed_dim=4), "both", [8], 1, "relu", embed_dim=4, seed=4)
    with torch.no_grad():
        q.dnn_layer.output_layer.bias.fill_(0.5)
        q.dnn_layer.output_layer.kernel.mul_(0.1)
    hid, dout = dnn_params(q.dnn_layer)
    pp = {"tables": tables_of(q.embed_layer), "dnn_hidden": hid, "dnn_out": dout,
          "outer_W": c(q.outer_product_layer.W)}
    loss = q.train_step((dense, ids), t, lr=0.3, return_loss=True)
    pp, ce = O.pnn_train_step(ids, t, pp, 0.3, mode="both")
    assert_scaled_close(loss, ce, what="PNN B=1 loss")
    assert_scaled_close(q.outer_product_layer.W, pp["outer_W"], what="PNN B=1 outer W")
    # DIN (T = 1)
    cols, behaviour = din_columns(1, 4, item_vocab=6, cate_vocab=3, user_vocab=5)
    inputs = din_inputs(np.random.default_rng(2), cols, behaviour, 3, 1)
    inputs = {k_: v_[:1] for k_, v_ in inputs.items()}
    dm = rs.DIN(cols, behaviour, att_hidden_units=(4,), dnn_hidden_units=(4,), seed=5)
    dm(inputs)
    before = _flat_params(_din_train_params(dm))
    pd = _din_train_params(dm)
    dm.train_step(inputs, t, lr=0.3)
    sf = [f_["feat"] for f_ in cols[1]]
    pd, _ = O.din_train_step(inputs, t, pd, [f_["feat"] for f_ in cols[0]], sf, [x for x in sf if x in behaviour], 0.3)
    got, ref = _flat_params(_din_train_params(dm)), _flat_params(pd)
    for name in ref:
        assert_scaled_close(got[name], ref[name], rtol=1e-4, what=f"DIN B=1 {name}")
