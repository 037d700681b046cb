"""Batched answers (BASELINE configs[2]: many keys against one shard pass): every key of a batch
must get exactly the answer it gets alone -- the oracle's answer on the same key and shard --
for every keys-per-pass grouping, ragged last groups, multi-round keys, partitions and the
byzantine flag; at full size the 2-party PIR property holds for every key of the batch."""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pir():
    import erasurecodedpir_amd as pir
    pir.load()
    return pir


def _keys(p, n, nq, idxs, rng):
    fcw = O.final_cw(p, nq, 1)
    out = []
    for idx in idxs:
        seeds = rng.integers(0, 256, 16 * p, dtype=np.uint8).tobytes()
        out.append(O.gen_keys(n, int(idx), fcw, p, nq, seeds))
    return out  # [key index][party]


BATCH_SHAPES = [  # (p, n, efs, nq, num_keys, keys per pass; 0 = automatic)
    (2, 12, 256, 1, 13, 0), (2, 10, 96, 1, 8, 16), (2, 11, 1024, 1, 5, 4), (2, 9, 1, 1, 3, 2),
    (3, 11, 100, 3, 5, 0), (3, 10, 48, 2, 9, 8), (5, 9, 48, 4, 7, 4), (8, 10, 64, 5, 3, 2),
    (8, 10, 64, 5, 3, 0), (2, 13, 4096, 1, 4, 8), (17, 8, 40, 16, 2, 0), (9, 9, 32, 1, 17, 16),
    # more keys than one frontier launch takes (256): frontiers in several launches
    (2, 6, 16, 1, 300, 0), (3, 7, 24, 2, 270, 4),
    # 8 share bytes per record and records >= 256 B: k_scan_t over key-major shares (1, 2 and
    # 4 bytes per key; ragged last groups)
    (3, 12, 256, 2, 9, 0), (5, 12, 512, 4, 5, 0), (4, 11, 320, 3, 3, 0), (2, 14, 768, 1, 11, 8),
]


@pytest.mark.parametrize("shape", BATCH_SHAPES, ids=lambda s: "p%d_n%d_efs%d_nq%d_k%d_g%d" % s)
def test_batch_vs_oracle(pir, shape):
    p, n, efs, nq, nk, g = shape
    rng = np.random.default_rng(hash(shape) & 0xFFFF)
    idxs = rng.integers(0, 1 << n, nk)
    keys = _keys(p, n, nq, idxs, rng)
    shard = rng.integers(0, 256, (1 << n) * efs, dtype=np.uint8)
    party = int(rng.integers(0, p))
    with pir.Engine(p, party + 1, n, efs, nq) as e:
        e.set_shard(shard)
        e.batch_group = g
        got = e.answer_batch([k[party] for k in keys])
        single = e.answer(keys[-1][party])
    assert got.shape == (nk, nq, efs)
    for q in range(nk):
        want = O.answer(p, party + 1, n, efs, nq, keys[q][party], shard)
        assert np.array_equal(got[q], want), q
    assert np.array_equal(got[-1], single)


def test_batch_empty_and_single(pir):
    p, n, efs, nq = 2, 8, 64, 1
    rng = np.random.default_rng(5)
    keys = _keys(p, n, nq, [17], rng)
    shard = rng.integers(0, 256, (1 << n) * efs, dtype=np.uint8)
    with pir.Engine(p, 1, n, efs, nq) as e:
        e.set_shard(shard)
        assert e.answer_batch([]).shape == (0, nq, efs)
        one = e.answer_batch([keys[0][0]])
    assert np.array_equal(one[0], O.answer(p, 1, n, efs, nq, keys[0][0], shard))


def test_batch_partitions_xor_to_full(pir):
    p, n, efs, nq, nk = 2, 12, 256, 1, 6
    rng = np.random.default_rng(11)
    keys = [k[0] for k in _keys(p, n, nq, rng.integers(0, 1 << n, nk), rng)]
    shard = rng.integers(0, 256, ((1 << n), efs), dtype=np.uint8)
    with pir.Engine(p, 1, n, efs, nq) as e:
        e.set_shard(shard)
        full = e.answer_batch(keys)
    acc = np.zeros_like(full)
    rows = (1 << n) >> 2
    for part in range(4):
        with pir.Engine(p, 1, n, efs, nq, log_num_partitions=2, partition_index=part) as e:
            e.set_shard(shard[part * rows:(part + 1) * rows])
            acc ^= e.answer_batch(keys)
    assert np.array_equal(acc, full)


def test_batch_byzantine_random(pir):
    p, n, efs, nq = 2, 6, 64, 1
    keys = pir.gen_keys(n, 3, p, nq)
    with pir.Engine(p, 1, n, efs, nq, is_byzantine=True) as e:
        a = e.answer_batch([keys[0]] * 4)
    assert a.shape == (4, nq, efs) and not np.array_equal(a[0], a[1])


def test_batch_pir_property_full_size(pir):
    """configs[2] shape scaled to 2^20 x 256 B, 32 keys: per key ans1 ^ ans2 = finalCW * record."""
    p, nq, n, efs, nk = 2, 1, 20, 256, 32
    fcw = O.final_cw(p, nq, 1)
    rng = np.random.default_rng(3)
    idxs = [int(i) for i in rng.integers(0, 1 << n, nk)]
    keys = [pir.gen_keys(n, i, p, nq, fcw=fcw) for i in idxs]
    ans = []
    recs = None
    for party in range(p):
        with pir.Engine(p, party + 1, n, efs, nq) as e:
            e.fill_shard_random(0xBA7C4)
            recs = [e.shard_row(i) for i in idxs]
            ans.append(e.answer_batch([k[party] for k in keys]))
    table = np.array([O.gf_mul(int(fcw[0]), x) for x in range(256)], np.uint8)
    for q in range(nk):
        assert np.array_equal(ans[0][q][0] ^ ans[1][q][0], table[recs[q]]), q


# ------------------------------------------------------------------ the depth-first leaf stage
# k_leaves (pir_leaves.hip) takes every leaf-converting stage of 4-5 levels: one input node per
# lane, 4-table AES with byte-trimmed control-bit (1/2/4 bytes for p = 2-5 / 6-9 / 10-17) and
# leaf blocks.  Its answers must equal the oracle's for every share width (nrp 1-16), party
# count class and leaf-stage depth, alone and batched.
LEAF_SHAPES = [  # (p, n, nq)
    (2, 16, 1), (3, 17, 2), (5, 15, 4), (8, 16, 5), (9, 14, 8), (12, 15, 9), (17, 14, 16),
]


@pytest.mark.parametrize("shape", LEAF_SHAPES, ids=lambda s: "p%d_n%d_nq%d" % s)
def test_leaf_stage_eval_all_vs_oracle(pir, shape):
    p, n, nq = shape
    rng = np.random.default_rng(hash(shape) & 0xFFFF)
    idx = int(rng.integers(0, 1 << n))
    seeds = rng.integers(0, 256, 16 * p, dtype=np.uint8).tobytes()
    keys = O.gen_keys(n, idx, O.final_cw(p, nq, 1), p, nq, seeds)
    for party in sorted({0, p - 1}):
        with pir.Engine(p, party + 1, n, 16, nq) as e:
            got = e.eval_all(keys[party])
        assert np.array_equal(got, O.eval_all(p, party, n, keys[party], nq)), party


@pytest.mark.parametrize("klast", [4, 5])
@pytest.mark.parametrize("p,n,efs,nq,nk,g", [(2, 15, 256, 1, 10, 8), (8, 14, 64, 5, 3, 2),
                                             (12, 13, 32, 9, 2, 1), (3, 14, 48, 2, 9, 0)])
def test_batch_leaf_depth_vs_oracle(pir, monkeypatch, klast, p, n, efs, nq, nk, g):
    monkeypatch.setenv("PIR_BATCH_KLAST", str(klast))
    rng = np.random.default_rng(1000 * klast + p)
    keys = _keys(p, n, nq, rng.integers(0, 1 << n, nk), rng)
    shard = rng.integers(0, 256, (1 << n) * efs, dtype=np.uint8)
    party = p - 1
    with pir.Engine(p, party + 1, n, efs, nq) as e:
        e.set_shard(shard)
        e.batch_group = g
        got = e.answer_batch([k[party] for k in keys])
    for q in range(nk):
        assert np.array_equal(got[q], O.answer(p, party + 1, n, efs, nq, keys[q][party], shard)), q


@pytest.mark.parametrize("p,n,efs,nq", [(2, 18, 256, 1), (3, 17, 512, 2), (5, 16, 1024, 4)])
def test_batch_key_major_equals_interleaved(pir, monkeypatch, p, n, efs, nq):
    """The key-major share layout with packed 16-byte leaf stores (k_scan_t groups) and the
    interleaved per-record layout with one store per leaf ($PIR_BATCH_KMAJOR=0,
    $PIR_LEAF_PACK=0) answer every key of a batch the same; spot keys against the oracle."""
    rng = np.random.default_rng(n * 13 + p)
    nk = 19
    keys = [k[0] for k in _keys(p, n, nq, rng.integers(0, 1 << n, nk), rng)]
    out = {}
    for mode, env in (("kmaj", {}), ("inter", {"PIR_BATCH_KMAJOR": "0", "PIR_LEAF_PACK": "0"})):
        for k in ("PIR_BATCH_KMAJOR", "PIR_LEAF_PACK"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        with pir.Engine(p, 1, n, efs, nq) as e:
            e.fill_shard_random(0x4B4D)
            out[mode] = e.answer_batch(keys)
            if mode == "kmaj":
                shard = e.get_shard()
    assert np.array_equal(out["kmaj"], out["inter"])
    for q in (0, nk - 1):
        assert np.array_equal(out["kmaj"][q], O.answer(p, 1, n, efs, nq, keys[q], shard.reshape(-1))), q
