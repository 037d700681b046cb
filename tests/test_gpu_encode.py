"""Server setup on the GPU: the erasure-coded shard (encode across files, client.cpp:70-97)
computed by k_encode_across equals the oracle restatement (itself pinned to the reference's
shard hashes in tests/golden/e2e.json), from explicit files and from the reference's synthetic
database; and the configs[4] pipeline end to end -- p = 8 servers (k=5, r=2) each encoding its
own shard on the GPU, answering, two servers dropped, client decode -- recovers the record."""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pir():
    import erasurecodedpir_amd as pir
    pir.load()
    return pir


@pytest.mark.parametrize("L,f,k,r", [(10, 8, 1, 1), (10, 8, 2, 1), (12, 16, 4, 2), (12, 16, 5, 2),
                                     (11, 100, 3, 1), (13, 1024, 5, 2), (9, 48, 16, 0)])
def test_encode_synthetic_matches_oracle(pir, L, f, k, r):
    p, n, efs, nq, _ = O.tree_sizes(L, f, k, r)
    files = O.synthetic_db(L, f)
    for party in sorted({1, p, (p + 1) // 2}):
        want = O.encode_across(L, f, k, p, party, files).reshape(1 << n, f)
        with pir.Engine(p, party, n, efs, nq) as e:
            e.encode_across(1 << L, k)
            assert np.array_equal(e.get_shard(), want), party
            e.encode_across(1 << L, k, files=files.reshape(1 << L, f))
            assert np.array_equal(e.get_shard(), want), party


def test_encode_reference_shard_hashes(pir):
    """Straight against the reference's own shard bytes (sha256 per party, e2e.json)."""
    for case in O.golden("e2e.json")["cases"]:
        L, f, k = case["L"], case["f"], case["k"]
        p, n, efs, nq = case["p"], case["n"], case["efs"], case["nq"]
        for party in range(1, p + 1):
            with pir.Engine(p, party, n, efs, nq) as e:
                e.encode_across(1 << L, k)
                assert O.sha(e.get_shard()) == case["shard_sha256"][party - 1], (case["L"], party)


def test_encode_random_files_and_partitions(pir):
    L, f, k, r = 14, 200, 4, 2
    p, n, efs, nq, _ = O.tree_sizes(L, f, k, r)
    rng = np.random.default_rng(3)
    files = rng.integers(0, 256, ((1 << L), f), dtype=np.uint8)
    want = O.encode_across(L, f, k, p, 2, files.reshape(-1)).reshape(1 << n, f)
    G = 2
    rows = (1 << n) >> G
    for part in range(1 << G):
        with pir.Engine(p, 2, n, efs, nq, log_num_partitions=G, partition_index=part) as e:
            e.encode_across(1 << L, k, files=files)
            assert np.array_equal(e.get_shard(), want[part * rows:(part + 1) * rows]), part


@pytest.mark.parametrize("L,f,k,r,drop", [(18, 1024, 5, 2, (2, 6)), (15, 256, 6, 1, (0,)),
                                          (17, 512, 4, 3, (1, 4, 5))])
def test_configs4_pipeline_end_to_end(pir, L, f, k, r, drop):
    """configs[4] shape (scaled): every server encodes its shard on the GPU, answers its key;
    R servers are dropped and the client decodes the record from the other answers."""
    from erasurecodedpir_amd import server as S
    S.setSystemParams(L, f, 1, k, r, 0, 1, 0, 0)
    prm = S.params()
    p, n, nq, efs = prm["NUM_PARTIES"], prm["LOG_NUM_ENCODED_FILES"], prm["NUM_ROUNDS"], prm["ENCODED_FILE_SIZE_BYTES"]
    encdb = -(-(1 << L) // k)
    row = encdb // 3 + 11  # a row of the encoded database = the index the client asks for
    keys = pir.gen_keys(n, row, p, nq, fcw=pir.final_cw(p, nq, 1))
    answers = []
    for party in range(1, p + 1):
        with pir.Engine(p, party, n, efs, nq) as e:
            e.encode_across(1 << L, k)
            answers.append(e.answer(keys[party - 1]))
    er = [0 if i in drop else 1 for i in range(p)]
    kept = np.stack([answers[i] for i in range(p) if er[i]])
    dec = S.assembleDPFTreeQueryResponses(er, kept)
    # the query for encoded row `row` decodes to file `row` (client.cpp:211-268)
    assert np.array_equal(dec, O.synthetic_db(L, f).reshape(-1, f)[row])
