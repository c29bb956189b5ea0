"""CPU: host-side logic of the Keras-compatible layers/models (construction,
Keras-shaped weights and names, initialiser statistics, error behaviour).
Modules are built on the CPU device; no kernel is launched."""
import numpy as np
import pytest
import torch

from recommender_system_amd import (DCN, PNN, Attention, CrossLayer, DeepFM, Dense, DNNLayer, EmbedLayer, FMLayer)
from tests.helpers import criteo_columns

DEV = "cpu"


def test_embed_layer_layout_and_names():
    cols = criteo_columns([5, 7, 3])[1]
    e = EmbedLayer(cols, k=4, device=DEV, seed=0)
    assert e.table.shape == (15, 4) and e.row_offsets == [0, 5, 12]
    assert e.field_table(1).shape == (7, 4)
    w = e.keras_weights()
    assert list(w) == ["embedding_0/embeddings", "embedding_1/embeddings", "embedding_2/embeddings"]
    assert float(e.table.abs().max()) <= 0.05  # Keras Embedding U(-0.05, 0.05)
    new = {k: np.full(v.shape, i, np.float32) for i, (k, v) in enumerate(w.items())}
    e.set_keras_weights(new)
    assert float(e.field_table(2).mean()) == 2.0


def test_embed_layer_default_k_is_8_and_ignores_embed_dim():
    cols = criteo_columns([5, 7], embed_dim=32)[1]
    assert EmbedLayer(cols, device=DEV).k == 8  # layer/core.py:268-271


def test_fm_layer_keras_shapes_and_init():
    fm = FMLayer(10, device=DEV, seed=1, input_dim=429)
    w = fm.keras_weights()
    assert w["w0"].shape == (1,) and w["w1"].shape == (429, 1) and w["v"].shape == (429, 10)
    assert float(w["w0"]) == 0.0
    assert abs(float(w["v"].std()) - 0.05) < 0.005  # random_normal_initializer stddev 0.05


def test_cross_layer_weights():
    c = CrossLayer(3, device=DEV, seed=2, input_dim=20)
    w = c.keras_weights()
    assert sorted(w) == ["b0", "b1", "b2", "w0", "w1", "w2"]
    assert all(v.shape == (20, 1) for v in w.values())


def test_dense_glorot_and_prelu_alpha():
    d = Dense(256, "prelu", device=DEV, seed=3, input_dim=429)
    lim = np.sqrt(6 / (429 + 256))
    assert float(d.kernel.abs().max()) <= lim and d.kernel.shape == (429, 256)
    assert float(d.alpha.abs().sum()) == 0.0 and d.alpha.shape == (256,)


def test_dnn_layer_structure():
    dnn = DNNLayer([256, 128, 64], 1, "relu", device=DEV, seed=4)
    dnn.build(429)
    shapes = [tuple(v.shape) for v in dnn.keras_weights().values()]
    assert shapes == [(429, 256), (256,), (256, 128), (128,), (128, 64), (64,), (64, 1), (1,)]


def test_models_construct_with_reference_signatures():
    cols = criteo_columns(np.full(26, 50))
    m = DeepFM(cols, 10, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=16, device=DEV)
    assert m.fm.v.shape == (13 + 26 * 16, 10)
    m2 = DCN(cols, [256, 128, 64], 1, "relu", layer_num=3, device=DEV, embed_dim=16)
    assert m2.output_layer.kernel.shape == (429 + 1, 1)
    m3 = PNN(cols, "inner", [256, 128, 64], 1, device=DEV, embed_dim=16)
    assert m3.width == 26 * 16 + 325


def test_pnn_mode_errors():
    cols = criteo_columns([5] * 4)
    with pytest.raises(ValueError, match="Please choice mode"):
        PNN(cols, "bogus", [8], 1, device=DEV)
    m = PNN(cols, "both", [8], 1, device=DEV, embed_dim=4)  # outer/both are built (OuterProductLayer)
    assert m.width == 4 * 4 + 2 * 6 and tuple(m.outer_product_layer.W.shape) == (4, 6, 4)
    with pytest.raises(NotImplementedError):
        PNN(cols, "inner", [8], 1, use_fgcnn=True, device=DEV)


def test_attention_prelu_alpha_shape_is_T_by_h():
    att = Attention((80, 40), "prelu", device=DEV, seed=5)
    att.build(100, 8)
    w = att.keras_weights()
    assert w["dense_0/kernel"].shape == (32, 80) and w["dense_0/prelu/alpha"].shape == (100, 80)
    assert w["dense_1/prelu/alpha"].shape == (100, 40) and w["out/kernel"].shape == (40, 1)
    with pytest.raises(ValueError):
        Attention((80, 40), "sigmoid", device=DEV)


def test_attention_dice_has_no_dense():
    att = Attention((80, 40), "dice", device=DEV)
    att.build(10, 8)
    w = att.keras_weights()
    assert not any(k.startswith("dense_") for k in w)
    assert w["dice_0/dice_alpha"].shape == (32,) and w["out/kernel"].shape == (32, 1)
