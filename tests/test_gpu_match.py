"""GPU parity of the descriptor matcher (match_points, src/my_utilities.h:70-120) against the
CPU oracle.  Integer/index work: best_idx, best/second distances and the accept flag must be
BIT-IDENTICAL (both sum the squared differences in dimension order with FP contraction off)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


_MODE = {"kernel": "mfma"}


@pytest.fixture(params=["mfma", "exact", "accept_only"], autouse=True)
def matcher_kernel(request, monkeypatch):
    """Every test runs on three forms, selected by picp_match_batch_form's explicit argument: the
    MFMA pre-filter (the default "full" form) and the exact scan ("exact") must give the oracle's
    bits; the accept-only radius form the VO sequence runs ("accept_only") must give the oracle's
    accept flags, and its best index and best distance wherever a query is accepted."""
    import functools

    import picp_amd
    form = {"mfma": "full", "exact": "exact", "accept_only": "accept_only"}[request.param]
    monkeypatch.setattr(picp_amd, "match_points", functools.partial(_MATCH[0], form=form))
    monkeypatch.setattr(picp_amd, "match_points_batch", functools.partial(_MATCH[1], form=form))
    _MODE["kernel"] = request.param
    return request.param


def _unpatched():
    import picp_amd
    return picp_amd.match_points, picp_amd.match_points_batch


_MATCH = _unpatched()


def _eq(got, ref):
    if _MODE["kernel"] == "accept_only":
        np.testing.assert_array_equal(got["accepted"], ref["accepted"], err_msg="accepted")
        acc = ref["accepted"].astype(bool)
        for k in ("best_idx", "best_dist"):
            np.testing.assert_array_equal(got[k][acc], ref[k][acc], err_msg=k)
        return
    for k in ("best_idx", "best_dist", "second_dist", "accepted"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


def _sets(rng, n1, n2, dim, frac_true=0.6):
    d2 = rng.random((n2, dim), dtype=np.float32)
    nt = min(int(n1 * frac_true), n2)
    d1 = rng.random((n1, dim), dtype=np.float32)
    if nt:
        d1[:nt] = d2[rng.choice(n2, nt, replace=False)] + rng.normal(0, 0.01, (nt, dim)).astype(np.float32)
    return d1, d2


@pytest.mark.parametrize("n1,n2,dim", [(1, 1, 10), (37, 300, 10), (1000, 2000, 10), (513, 257, 10),
                                       (300, 700, 7), (200, 900, 32), (5000, 1, 10)])
def test_match_matches_oracle(native, oracle, n1, n2, dim):
    rng = np.random.default_rng(n1 * 31 + n2 + dim)
    d1, d2 = _sets(rng, n1, n2, dim)
    if n2 > 3:
        d2[2] = d2[3]  # exact tie: lower index wins
    _eq(native.match_points(d1, d2), oracle.match_points(d1, d2))


def test_match_reference_data_frames(native, oracle, vo):
    """data/: each measurement frame against the map, and consecutive frames against each other
    (the two match_points call sites of exec/icp_test.cpp)."""
    for k in range(0, 20):
        f = vo.frame(k)
        _eq(native.match_points(f["desc"], vo.world_desc), oracle.match_points(f["desc"], vo.world_desc))
        g = vo.frame(k + 1)
        _eq(native.match_points(f["desc"], g["desc"]), oracle.match_points(f["desc"], g["desc"]))


def test_match_batch_ragged(native, oracle):
    rng = np.random.default_rng(3)
    sizes = [(0, 5), (4, 0), (300, 1000), (1, 1), (700, 50), (0, 0), (2049, 333)]
    d1s, d2s = zip(*[_sets(rng, a, b, 10) for a, b in sizes])
    outs = native.match_points_batch(list(d1s), list(d2s))
    for d1, d2, got in zip(d1s, d2s, outs):
        _eq(got, oracle.match_points(d1, d2))


def test_match_thresholds(native, oracle):
    rng = np.random.default_rng(11)
    d1, d2 = _sets(rng, 800, 800, 10)
    for dt, rt in [(0.2, 0.8), (1e9, 1.0), (0.0, 0.8), (0.05, 0.3)]:
        _eq(native.match_points(d1, d2, dt, rt), oracle.match_points(d1, d2, dt, rt))


def test_match_empty_and_errors(native):
    d = np.ones((4, 10), np.float32)
    got = native.match_points(d, np.zeros((0, 10), np.float32))
    assert (got["best_idx"] == -1).all() and not got["accepted"].any()
    assert len(native.match_points(np.zeros((0, 10), np.float32), d)["best_idx"]) == 0
    with pytest.raises(Exception):
        native.match_points(np.ones((4, 33), np.float32), np.ones((4, 33), np.float32))


def test_match_large_norm_rows_and_whole_tiles(native, oracle):
    """Whole 256-row reference tiles and a partial last one; a reference and a query with
    |x|^2 > 60000 whose components are still inside fp16 range (the bound scales with the
    norms); a tie and a near match inside a tile; a batch of two problems."""
    rng = np.random.default_rng(17)
    d2 = rng.uniform(-1, 1, (3 * 256 + 77, 10)).astype(np.float32)
    d2[300] = 100.0                      # |r|^2 = 1e5, components inside fp16 range
    d2[600] = d2[601]                    # a tie inside a whole tile
    d1 = np.concatenate([d2[[5, 300, 600, 700, 770, 3 * 256 + 70]] + 0.0,
                         rng.uniform(-1, 1, (200, 10)).astype(np.float32),
                         np.full((1, 10), 90.0, np.float32)])    # |q|^2 = 81000
    d1[7] = d2[9] + 0.1                  # near match, |d| = 0.1
    _eq(native.match_points(d1, d2), oracle.match_points(d1, d2))
    batch = native.match_points_batch([d1, d1[:50]], [d2, d2[:300]])
    _eq(batch[0], oracle.match_points(d1, d2))
    _eq(batch[1], oracle.match_points(d1[:50], d2[:300]))


def test_match_adversarial_fallbacks(native, oracle):
    """The pre-filter's exits: exact duplicate references (ties, 0/0 ratio), a crowd of
    references inside one query's candidate window (more than 16 candidates -> full scan),
    components beyond fp16 range and non-finite ones (forced candidates / full scan)."""
    rng = np.random.default_rng(5)
    d2 = rng.uniform(-1, 1, (700, 10)).astype(np.float32)
    d2[10] = d2[11] = d2[500]                      # triple duplicate
    d2[600:660] = d2[600] + rng.normal(0, 1e-4, (60, 10)).astype(np.float32)  # 60 near-twins
    d2[50, 3] = 1e6                                # beyond fp16 range
    d2[51, 0] = np.nan
    d2[52, 9] = np.inf
    d1 = np.concatenate([d2[[10, 600, 601, 3, 50]] + 0.0, rng.uniform(-1, 1, (300, 10)).astype(np.float32)])
    d1[5, 2] = 7e4                                 # query beyond fp16 range
    d1[6, 1] = np.nan
    _eq(native.match_points(d1, d2), oracle.match_points(d1, d2))
    # large magnitudes everywhere (norms ~1e8): the bound scales with them
    big = (rng.uniform(-1, 1, (400, 10)) * 3e3).astype(np.float32)
    _eq(native.match_points(big[:150], big[150:], 1e9, 0.8), oracle.match_points(big[:150], big[150:], 1e9, 0.8))
    # tiny magnitudes (fp16 subnormals)
    tiny = (rng.uniform(-1, 1, (400, 10)) * 1e-5).astype(np.float32)
    _eq(native.match_points(tiny[:150], tiny[150:], 1.0, 0.8), oracle.match_points(tiny[:150], tiny[150:], 1.0, 0.8))


def test_match_batch_two_row_blocks(native, oracle, monkeypatch):
    """The matcher's two-row-block form (RB = 2, 64 queries per wave), what the C5 sequence runs:
    the accept-only form picks it by itself once n_problems x ceil(nq / 256) >= 4 x CUs (1024
    problems of 200 queries here); PICP_MATCH_RB=2 forces it on the other forms.  Exact ties and
    duplicated references (best = second, ratio 0/0 rejected) in every problem, problems of 1 and
    0 queries and an empty reference set mixed in."""
    if _MODE["kernel"] != "accept_only":
        monkeypatch.setenv("PICP_MATCH_RB", "2")
    rng = np.random.default_rng(2024)
    d1s, d2s = [], []
    for i in range(1024):
        n1, n2 = (200, 300) if i % 97 else (1 if i % 2 else 0, 0 if i % 194 else 40)
        d1, d2 = _sets(rng, n1, n2, 10, frac_true=0.7)
        if n2 > 8:
            d2[4] = d2[5]          # exact duplicate reference
            d2[7] = d2[6] + 0.0
            if n1 > 3:
                d1[2] = d2[4]      # a query sitting on the duplicate: distance 0 twice
                d1[3] = d2[6] + np.float32(1e-3)
        d1s.append(d1)
        d2s.append(d2)
    outs = native.match_points_batch(d1s, d2s)
    for d1, d2, got in zip(d1s, d2s, outs):
        _eq(got, oracle.match_points(d1, d2))


@pytest.mark.parametrize("rb", ["default", "2"])
@pytest.mark.parametrize("ksplit", ["1", "3", "5", "16"])
def test_match_reference_range_split(native, oracle, monkeypatch, ksplit, rb):
    """The reference-range split (picp_match_ksplit: few problems against many references, e.g.
    the VO world match of a few long segments): each range's top-2 is merged in range order
    (picp_match_merge_kernel).  PICP_MATCH_KSPLIT forces the range count; ranges are >= 1,024 rows,
    so 5,000 references make up to 5.  Exact duplicates on both sides of range boundaries (the
    lower index must win and second = best), a triple duplicate across three ranges, near-ties
    across a boundary, and a ragged batch with empty sets."""
    monkeypatch.setenv("PICP_MATCH_KSPLIT", ksplit)
    if rb != "default":  # two row blocks per wave with the split (the 8e world match's form since round 6)
        monkeypatch.setenv("PICP_MATCH_RB", rb)
    rng = np.random.default_rng(77)
    d2 = rng.uniform(-1, 1, (5000, 10)).astype(np.float32)
    d2[1024] = d2[1023]                                   # boundary of ranges 0 | 1
    d2[2048] = d2[4000] = d2[2047]                        # across ranges 1 | 2 | 3
    d2[3072] = d2[3071] + np.float32(1e-4)                # near-tie across 2 | 3
    d1 = np.concatenate([d2[[1023, 1024, 2047, 3071, 3072, 4999, 0]] + 0.0,
                         d2[rng.choice(5000, 600, replace=False)] + rng.normal(0, 0.01, (600, 10)).astype(np.float32),
                         rng.uniform(-1, 1, (300, 10)).astype(np.float32)])
    _eq(native.match_points(d1, d2), oracle.match_points(d1, d2))
    sizes = [(0, 5), (40, 0), (700, 5000), (1, 1), (0, 0), (300, 2100)]
    d1s, d2s = zip(*[_sets(rng, a, b, 10) for a, b in sizes])
    d1s, d2s = list(d1s), list(d2s)
    d1s[2], d2s[2] = d1[:700], d2
    for d1_, d2_, got in zip(d1s, d2s, native.match_points_batch(d1s, d2s)):
        _eq(got, oracle.match_points(d1_, d2_))


@pytest.mark.parametrize("ksplit", ["1", "3"])
def test_match_unsafe_tiles_two_row_blocks(native, oracle, monkeypatch, ksplit):
    """Tiles holding an unsafe reference (|x|^2 > 60000, beyond fp16 range, NaN) between whole safe
    tiles, at two row blocks per wave and with a range split: the accept-only form decides per
    tile between the folded test and the compare (the decision travels with the tile through LDS
    since round 6), the other forms take their own paths; the last tile is partial."""
    monkeypatch.setenv("PICP_MATCH_RB", "2")
    monkeypatch.setenv("PICP_MATCH_KSPLIT", ksplit)
    rng = np.random.default_rng(99)
    d2 = rng.uniform(-1, 1, (4 * 1024 + 37, 10)).astype(np.float32)
    d2[300] = 100.0                      # |r|^2 = 1e5 inside fp16 range (tile 1)
    d2[1500, 4] = 1e6                    # beyond fp16 range (tile 5)
    d2[2900, 0] = np.nan                 # non-finite (tile 11)
    d2[4100] = d2[4099]                  # a tie in the partial last tile
    d1 = np.concatenate([d2[[299, 301, 1499, 1501, 2899, 2901, 4099, 4100, 0]] + 0.0,
                         d2[rng.choice(len(d2), 300, replace=False)] + rng.normal(0, 0.01, (300, 10)).astype(np.float32),
                         rng.uniform(-1, 1, (200, 10)).astype(np.float32)])
    _eq(native.match_points(d1, d2), oracle.match_points(d1, d2))


def test_match_past_2_24_references(native, oracle):
    """A reference set past 2^24 rows: the candidate entries index 2^20 references per
    range, so picp_match_ksplit splits such a set into more than MM_KSPLIT_MAX (16) ranges rather
    than send every query to the O(nr) full scan.  64 queries x (2^24 + 4,099) references: exact
    copies of references in the first, a middle and the last range (one duplicated across two
    ranges: 0/0 ratio -> reject, the lower index first), near-copies and far queries; every output
    bit-exact in all three forms."""
    rng = np.random.default_rng(2024)
    n_r, dim = (1 << 24) + 4099, 10
    r = rng.uniform(-1, 1, (n_r, dim)).astype(np.float32)
    src = np.array([3, 1 << 20, (1 << 20) + 1, 5_000_000, 9_999_999, 1 << 24, n_r - 1, 12_345_678])
    r[(1 << 24) + 7] = r[9_999_999]  # a duplicate in another range
    q = np.concatenate([r[src], r[src] + rng.uniform(-3e-3, 3e-3, (len(src), dim)).astype(np.float32),
                        rng.uniform(-1, 1, (64 - 2 * len(src), dim)).astype(np.float32)])
    ref = oracle.match_points(q, r)
    assert ref["accepted"].sum() >= len(src) - 1 and not ref["accepted"][4]
    for form in ("full", "exact", "accept_only"):
        got = native.match_points_batch([q], [r], form=form)[0]
        acc = ref["accepted"]
        np.testing.assert_array_equal(got["accepted"].astype(bool), acc)
        np.testing.assert_array_equal(got["best_idx"][acc], ref["best_idx"][acc])
        if form != "accept_only":
            np.testing.assert_array_equal(got["best_idx"], ref["best_idx"])
            np.testing.assert_array_equal(got["best_dist"].view(np.uint32), ref["best_dist"].view(np.uint32))
            np.testing.assert_array_equal(got["second_dist"].view(np.uint32), ref["second_dist"].view(np.uint32))
