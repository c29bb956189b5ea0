"""GPU parity of the hand-written stable radix sort and int32 scan
(csrc/radix_sort.hip) against numpy: the grouping step of every row-sparse
scatter-add (rs_embedding_sgd, rs_fm_train_step, the dedup route beyond 4096
samples).  Bit-exact: the sort must equal a stable argsort by the low `bits`
bits of the key, values carried along; the scan must equal np.cumsum."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _sort(gpu, keys, vals, bits):
    from recommender_system_amd import _lib
    lib = _lib.lib()
    n = keys.size
    kin = torch.from_numpy(keys.view(np.int32)).to(gpu)
    vin = torch.from_numpy(vals.view(np.int32)).to(gpu)
    kout = torch.full_like(kin, -7)
    vout = torch.full_like(vin, -7)
    ws = torch.empty(max(int(lib.rs_sort_pairs_workspace_size(n)), 1), dtype=torch.uint8, device=gpu)
    kin0, vin0 = kin.clone(), vin.clone()
    _lib.check(lib.rs_sort_pairs_u32(kin.data_ptr(), vin.data_ptr(), kout.data_ptr(), vout.data_ptr(), n, bits,
                                     ws.data_ptr(), _lib.stream()), "rs_sort_pairs_u32")
    torch.cuda.synchronize()
    assert torch.equal(kin, kin0) and torch.equal(vin, vin0), "inputs modified"
    return kout.cpu().numpy().view(np.uint32), vout.cpu().numpy().view(np.uint32)


def _expect(keys, vals, bits):
    mask = np.uint64((1 << bits) - 1)
    order = np.argsort(keys.astype(np.uint64) & mask, kind="stable")
    return keys[order], vals[order]


@pytest.mark.parametrize("n,bits,span", [
    (1, 1, 2), (63, 7, 100), (4095, 12, 4000), (4096, 16, 60000), (4097, 20, 1 << 20),
    (106_496, 25, 26_000_000),      # one B 4096 x 26 batch of lookups, 26 x 1e6 rows
    (300_001, 32, 1 << 32),         # full-width keys, ragged last tile
    (1_703_936, 25, 26_000_000),    # B 65536 x 26: the scan-launch path (many tiles)
    (50_000, 9, 3),                 # very few distinct keys: long equal runs, stability
])
def test_sort_pairs_matches_stable_argsort(gpu, n, bits, span):
    rng = np.random.default_rng(n + bits)
    keys = rng.integers(0, span, size=n, dtype=np.uint64).astype(np.uint32)
    vals = np.arange(n, dtype=np.uint32)
    k, v = _sort(gpu, keys, vals, bits)
    ek, ev = _expect(keys, vals, bits)
    assert np.array_equal(k, ek) and np.array_equal(v, ev)


def test_sort_pairs_bad_keys_last_and_zipf(gpu):
    """The embedding SGD's layout: 0xffffffff marks a bad id and must land after
    every valid row (bits chosen with 2^bits > rows); Zipf-hot rows keep their
    lookups in order."""
    rng = np.random.default_rng(5)
    n, rows = 26 * 4096, 26_000_000
    keys = np.minimum(rng.zipf(1.05, size=n) - 1, rows - 1).astype(np.uint32)
    keys[rng.integers(0, n, 100)] = 0xFFFFFFFF
    vals = rng.permutation(n).astype(np.uint32)
    bits = int(np.ceil(np.log2(rows + 1)))
    k, v = _sort(gpu, keys, vals, bits)
    ek, ev = _expect(keys, vals, bits)
    assert np.array_equal(k, ek) and np.array_equal(v, ev)
    assert np.all(k[-100:] == 0xFFFFFFFF)


@pytest.mark.parametrize("n", [1, 17, 4096, 4097, 106_496, 1_000_003])
def test_inclusive_sum_matches_cumsum(gpu, n):
    from recommender_system_amd import _lib
    lib = _lib.lib()
    rng = np.random.default_rng(n)
    x = rng.integers(0, 3, size=n).astype(np.int32)
    xin = torch.from_numpy(x).to(gpu)
    out = torch.empty_like(xin)
    ws = torch.empty(int(lib.rs_inclusive_sum_workspace_size(n)), dtype=torch.uint8, device=gpu)
    _lib.check(lib.rs_inclusive_sum_i32(xin.data_ptr(), out.data_ptr(), n, ws.data_ptr(), _lib.stream()),
               "rs_inclusive_sum_i32")
    assert np.array_equal(out.cpu().numpy(), np.cumsum(x, dtype=np.int64).astype(np.int32))
    # in place
    _lib.check(lib.rs_inclusive_sum_i32(xin.data_ptr(), xin.data_ptr(), n, ws.data_ptr(), _lib.stream()),
               "rs_inclusive_sum_i32")
    assert np.array_equal(xin.cpu().numpy(), np.cumsum(x, dtype=np.int64).astype(np.int32))


def test_sort_and_scan_empty(gpu):
    from recommender_system_amd import _lib
    lib = _lib.lib()
    assert lib.rs_sort_pairs_u32(None, None, None, None, 0, 8, None, _lib.stream()) == 0
    assert lib.rs_inclusive_sum_i32(None, None, 0, None, _lib.stream()) == 0
