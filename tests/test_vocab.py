"""String-vocabulary kernels (csrc/vocab.hip) vs the exact host implementation of
tft.compute_and_apply_vocabulary semantics in mifx.transform.api."""
import numpy as np
import pytest

from mifx.ops import vocab as V
from mifx.transform import api as tft


def _column(n=50000, seed=0):
    rng = np.random.default_rng(seed)
    # Zipf-ish company names + payment types + empties/None/bytes/unicode (taxi-like string columns)
    base = [f"company_{i}" for i in range(3000)] + ["Cash", "Credit Card", "No Charge", "", "Dispute", "Ünïcødé"]
    p = 1.0 / np.arange(1, len(base) + 1) ** 1.1
    idx = rng.choice(len(base), size=n, p=p / p.sum())
    col = [base[i] for i in idx]
    col[::97] = [None] * len(col[::97])
    col[5::211] = [b"Cash"] * len(col[5::211])
    return col


def test_pack_strings_roundtrip():
    col = ["a", "", None, b"xyz", "Ünï"]
    buf, offs, get = V.pack_strings(col)
    assert offs.tolist()[0] == 0 and offs[-1] == len("axyzÜnï".encode())
    got = [bytes(buf[offs[i]:offs[i + 1]]).decode() for i in range(len(col))]
    assert got == ["a", "", "", "xyz", "Ünï"] == [get(i) for i in range(len(col))]


def test_pack_strings_arrow_zero_copy_matches_list():
    import pyarrow as pa

    col = ["a", None, "", "xyz", "Ünï"] * 3
    arr = pa.chunked_array([pa.array(col[:7]), pa.array(col[7:])])
    buf, offs, get = V.pack_strings(arr)
    got = [bytes(buf[offs[i]:offs[i + 1]]).decode() for i in range(len(col))]
    assert got == [c or "" for c in col] == [get(i) for i in range(len(col))]
    sl = pa.array(col).slice(3, 5)  # non-zero Arrow offset
    buf, offs, get = V.pack_strings(sl)
    assert [bytes(buf[offs[i]:offs[i + 1]]).decode() for i in range(5)] == [c or "" for c in col[3:8]]
    assert V.vocabulary(arr, device=None) == V.vocabulary(col, device=None)


def test_fnv_matches_transform_fingerprint():
    for s in ["", "a", "Credit Card", "Ünïcødé", "x" * 300]:
        assert V.fnv1a64(s.encode()) == tft.fingerprint64(s)


def test_host_vocabulary_matches_transform_api():
    col = _column(5000)
    with tft._phase("analyze", tft.TransformState()):
        ref = tft.vocabulary(col, top_k=1000)
    assert V.vocabulary(col, top_k=1000) == ref
    got = V.apply_vocabulary(col, ref, default_value=-1, num_oov_buckets=10)
    assert np.array_equal(got, tft.apply_vocabulary(col, ref, default_value=-1, num_oov_buckets=10))


def test_order_ties_by_token_descending():
    assert V.order_vocabulary(["a", "b", "c"], [2, 2, 5]) == ["c", "b", "a"]
    assert V.order_vocabulary(["a", "b", "c"], [2, 2, 5], top_k=2) == ["c", "b"]
    assert V.order_vocabulary(["a", "b", "c"], [1, 2, 5], frequency_threshold=2) == ["c", "b"]


@pytest.mark.gpu
def test_gpu_hash_matches_host():
    col = _column(20000, seed=1)
    got = V.hash_strings(col, device="cuda")
    ref = V.hash_strings(col, device=None)
    assert got.dtype == np.uint64 and np.array_equal(got, ref)


@pytest.mark.gpu
def test_gpu_count_and_vocabulary_match_host():
    col = _column(200000, seed=2)
    toks, counts = V.count_unique(col, device="cuda")
    ht, hc = V.count_unique(col, device=None)
    assert dict(zip(toks, counts)) == dict(zip(ht, hc))
    for top_k, thr in ((None, None), (1000, None), (50, 3)):
        assert V.vocabulary(col, top_k, thr, device="cuda") == V.vocabulary(col, top_k, thr, device=None)


@pytest.mark.gpu
@pytest.mark.parametrize("oov,default", [(10, -1), (0, -1), (0, 7)])
def test_gpu_apply_vocabulary_matches_host(oov, default):
    col = _column(100000, seed=3)
    vocab = V.vocabulary(col[:20000], top_k=1000)
    got = V.apply_vocabulary(col, vocab, default_value=default, num_oov_buckets=oov, device="cuda")
    ref = tft.apply_vocabulary(col, vocab, default_value=default, num_oov_buckets=oov)
    assert np.array_equal(got, ref)


@pytest.mark.gpu
def test_transform_api_uses_gpu_vocab_path(monkeypatch):
    """compute_and_apply_vocabulary inside analyze(device='cuda') routes through the HIP kernels
    and yields exactly the CPU result."""
    calls = []
    real = V.count_unique
    monkeypatch.setattr(V, "count_unique", lambda *a, **k: calls.append(k.get("device")) or real(*a, **k))
    col = np.array(_column(60000, seed=4), dtype=object)

    def fn(inputs):
        return {"c": tft.compute_and_apply_vocabulary(inputs["c"], top_k=1000, num_oov_buckets=10)}

    out_gpu, st_gpu = tft.analyze(fn, {"c": col}, device="cuda")
    out_cpu, st_cpu = tft.analyze(fn, {"c": col}, device=None)
    assert any(d is not None for d in calls)
    assert st_gpu.entries == st_cpu.entries
    assert np.array_equal(out_gpu["c"], out_cpu["c"])


@pytest.mark.gpu
def test_gpu_arrow_column_matches_host():
    import pyarrow as pa

    col = [v.decode() if isinstance(v, bytes) else v for v in _column(100000, seed=5)]
    arr = pa.chunked_array([pa.array(col[:40000]), pa.array(col[40000:])])
    vocab = V.vocabulary(arr, top_k=1000, device="cuda")
    assert vocab == V.vocabulary(col, top_k=1000, device=None)
    got = V.apply_vocabulary(arr, vocab, default_value=-1, num_oov_buckets=10, device="cuda")
    assert np.array_equal(got, tft.apply_vocabulary(col, vocab, default_value=-1, num_oov_buckets=10))
