"""RSCB batch files (include/rs_batchio.h, csrc/batchio.cpp) and the device
batch loader (the input producer's on-disk format).

CPU: write/read round trips are bit-exact (int32 and int64 ids, ids >= 2**24
that the reference's float-packed X cannot carry), bad ids and bad files are
rejected, and the file made from the bundled Criteo sample carries exactly the
reference's own preprocessing output (the rows of the committed
create_criteo_dataset('DeepFM') fixture, tests/golden/criteo_ref.npz).
GPU: DeviceBatchLoader's batches equal the file's rows and drive the fused
kernel to the same logits as host-fed input.
"""
import os

import numpy as np
import pytest

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SAMPLE = os.path.join(G, "criteo_train_1w.txt.gz")


def _rows(rng, N, vocab, id_dtype):
    dense = rng.random((N, 13)).astype(np.float32)
    ids = np.stack([rng.integers(0, v, N) for v in vocab], 1).astype(id_dtype)
    labels = rng.integers(0, 2, N).astype(np.float32)
    return dense, ids, labels


@pytest.mark.parametrize("id_dtype", [np.int32, np.int64])
def test_roundtrip_bit_exact(tmp_path, id_dtype):
    from recommender_system_amd.batchio import RSCBFile, write_criteo
    rng = np.random.default_rng(1)
    vocab = rng.integers(1, 5000, 26)
    vocab[3] = 40_000_000 if id_dtype == np.int32 else 3_000_000_000  # ids >= 2**24 (> int32 for int64)
    dense, ids, labels = _rows(rng, 1001, vocab, id_dtype)
    ids[0, 3] = vocab[3] - 1
    p = write_criteo(tmp_path / "a.rscb", dense, ids, labels, vocab, id_dtype=id_dtype)
    with RSCBFile(p) as f:
        assert (f.n_rows, f.n_dense, f.n_sparse) == (1001, 13, 26)
        np.testing.assert_array_equal(f.field_vocab, vocab)
        np.testing.assert_array_equal(f.field_offsets, np.concatenate([[0], np.cumsum(vocab)[:-1]]))
        d2, i2, l2 = f.read()
        np.testing.assert_array_equal(d2, dense)
        np.testing.assert_array_equal(i2, ids)
        np.testing.assert_array_equal(l2, labels)
        d3, i3, _ = f.read(500, 17)
        np.testing.assert_array_equal(i3, ids[500:517])
        np.testing.assert_array_equal(d3, dense[500:517])
        with pytest.raises(Exception, match="outside"):
            f.read(1000, 2)
    # float32-packed ids (the reference's X) lose this id; RSCB keeps it
    assert float(np.float32(ids[0, 3])) != ids[0, 3] or vocab[3] < 2 ** 24


def test_rejects_bad_ids_and_files(tmp_path):
    from recommender_system_amd._lib import RSError
    from recommender_system_amd.batchio import RSCBFile, write_criteo
    rng = np.random.default_rng(2)
    vocab = np.full(26, 10)
    dense, ids, labels = _rows(rng, 5, vocab, np.int32)
    ids[2, 7] = 10
    with pytest.raises(RSError, match="outside"):
        write_criteo(tmp_path / "bad.rscb", dense, ids, labels, vocab)
    (tmp_path / "junk").write_bytes(b"x" * 5000)
    with pytest.raises(OSError, match="bad RSCB header"):
        RSCBFile(tmp_path / "junk")
    with pytest.raises(OSError, match="cannot open"):
        RSCBFile(tmp_path / "missing")
    empty = write_criteo(tmp_path / "empty.rscb", dense[:0], ids[:0], labels[:0], vocab)
    with RSCBFile(empty) as f:
        assert f.n_rows == 0
    # crafted headers: n_rows whose section sizes wrap uint64, a misaligned
    # section offset, a dense section overlapping the header page
    ids[2, 7] = 9
    good = write_criteo(tmp_path / "good.rscb", dense, ids, labels, vocab)
    raw = bytearray(open(good, "rb").read())
    import struct
    for field_off, value in [(24, (1 << 64) // (13 * 4) + 1), (32, 4096 + 4), (32, 0)]:
        b = bytearray(raw)
        struct.pack_into("<Q", b, field_off, value)  # 24: n_rows, 32: off_dense
        (tmp_path / "crafted").write_bytes(bytes(b))
        with pytest.raises(OSError, match="bad RSCB header"):
            RSCBFile(tmp_path / "crafted")


def test_bundled_sample_matches_reference_preprocessing(tmp_path):
    """RSCB from the bundled Criteo sample == the reference's own
    create_criteo_dataset('DeepFM') rows (committed fixture) — dense as the
    model's float32 cast, ids exact — and its vocab == features_dict's."""
    from recommender_system_amd.batchio import RSCBFile, criteo_txt_to_rscb
    ref = dict(np.load(os.path.join(G, "criteo_ref.npz")))
    p = criteo_txt_to_rscb(SAMPLE, tmp_path / "criteo.rscb")
    with RSCBFile(p) as f:
        dense, ids, labels = f.read()
        np.testing.assert_array_equal(f.field_vocab, ref["vocab"])
    X = ref["deepfm_X_train"]  # rows of the reference's split, in split order
    key = {tuple(r): i for i, r in enumerate(np.concatenate([dense, ids.astype(np.float32)], 1).tolist())}
    want = np.concatenate([X[:, :13].astype(np.float32), X[:, 13:].astype(np.float32)], 1)
    idx = [key.get(tuple(r)) for r in want.tolist()]
    assert all(i is not None for i in idx), "a reference row is missing from the RSCB file"
    np.testing.assert_array_equal(ids[idx], X[:, 13:].astype(np.int64))
    np.testing.assert_array_equal(labels[idx], ref["deepfm_y_train"].astype(np.float32))


@pytest.mark.gpu
def test_device_loader_feeds_fused_kernel(gpu, tmp_path):
    import torch

    import recommender_system_amd as rs
    from recommender_system_amd.batchio import DeviceBatchLoader, write_criteo
    from tests.helpers import criteo_columns
    rng = np.random.default_rng(3)
    vocab = rng.integers(2, 3000, 26)
    dense, ids, labels = _rows(rng, 1000, vocab, np.int32)
    p = write_criteo(tmp_path / "b.rscb", dense, ids, labels, vocab)
    m = rs.DeepFM(criteo_columns(vocab, embed_dim=16), 10, 1e-4, 1e-4, [64], 1, "relu", embed_dim=16, seed=1)
    B = 256
    seen = 0
    outs = []
    for d, i, lab in DeviceBatchLoader(p, B, depth=3):
        n = d.shape[0]
        np.testing.assert_array_equal(i.cpu().numpy(), ids[seen:seen + n])
        np.testing.assert_array_equal(lab.cpu().numpy(), labels[seen:seen + n])
        outs.append(m.fm_logit((d, i)).clone())
        seen += n
    assert seen == 1000 and len(outs) == 4
    ref = m.fm_logit((torch.as_tensor(dense, device=gpu), torch.as_tensor(ids, device=gpu)))
    np.testing.assert_array_equal(torch.cat(outs).cpu().numpy(), ref.cpu().numpy())
