"""Retrieval on CPU tensors (SURVEY §4.2 "Retrieval tests"): FlatIndex == brute-force torch.topk
(ip and l2), IVF with nprobe == nlist is exact, IVF recall on a clustered corpus, save/load round
trips, chunking, and the batched encoder (order-independent, unit-norm, dedup map).

The reference declares a vector store (README.md:28, "ChromaDB, FAISS") but implements none."""
import pytest
import torch

from rag_tl_domainllm_optimizer_amd.retrieval import FlatIndex, IVFIndex
from rag_tl_domainllm_optimizer_amd.retrieval.chunking import chunk_documents, chunk_text
from rag_tl_domainllm_optimizer_amd.retrieval.index import load_index


def _clustered(n=2000, d=32, centers=16, seed=0):
    g = torch.Generator().manual_seed(seed)
    c = torch.nn.functional.normalize(torch.randn(centers, d, generator=g), dim=-1)
    lab = torch.randint(0, centers, (n,), generator=g)
    x = c[lab] + 0.15 * torch.randn(n, d, generator=g)
    return torch.nn.functional.normalize(x, dim=-1)


@pytest.mark.parametrize("metric", ["ip", "l2"])
def test_flat_matches_bruteforce(metric):
    x = _clustered(500, 24)
    q = _clustered(20, 24, seed=3)
    idx = FlatIndex(24, metric)
    idx.add(x[:300])
    idx.add(x[300:], ids=torch.arange(1000, 1200))
    v, ids = idx.search(q, 5)
    all_ids = torch.cat([torch.arange(300), torch.arange(1000, 1200)])
    if metric == "ip":
        rv, ri = torch.topk(q @ x.t(), 5, dim=-1)
    else:
        rv, ri = torch.topk(-(torch.cdist(q, x) ** 2), 5, dim=-1)
        rv = -rv
    torch.testing.assert_close(v, rv, rtol=1e-4, atol=1e-4)
    assert torch.equal(ids, all_ids[ri])


def test_ivf_full_probe_is_exact_and_recall():
    x = _clustered(2000, 32)
    q = _clustered(40, 32, seed=5)
    flat = FlatIndex(32)
    flat.add(x)
    _, fi = flat.search(q, 10)
    ivf = IVFIndex(32, nlist=16, nprobe=16)
    ivf.train(x, niter=5)
    ivf.add(x)
    assert ivf.ntotal == 2000
    # the list offsets partition the database
    off = ivf.offsets.long()
    assert int(off[0]) == 0 and int(off[-1]) == 2000 and bool((off[1:] >= off[:-1]).all())
    _, ii = ivf.search(q, 10)
    assert torch.equal(torch.sort(ii, -1).values, torch.sort(fi, -1).values)
    # fewer probes: recall@10 stays high on a clustered corpus
    _, ip = ivf.search(q, 10, nprobe=4)
    hits = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(ip, fi))
    assert hits / fi.numel() >= 0.8


@pytest.mark.parametrize("metric", ["ip", "l2"])
def test_ivf_incremental_add_and_l2(metric):
    """Adding in pieces (several list re-layouts) gives the same search results as one add; with
    nprobe == nlist the IVF search is exact for both metrics."""
    x = _clustered(1500, 16, seed=2) * (1.0 if metric == "ip" else 3.0)
    q = _clustered(30, 16, seed=7) * (1.0 if metric == "ip" else 3.0)
    one = IVFIndex(16, nlist=12, metric=metric, nprobe=12)
    one.train(x, niter=4)
    one.add(x)
    inc = IVFIndex(16, nlist=12, metric=metric, nprobe=12)
    inc.train(x, niter=4)
    for s in (0, 7, 300, 301, 900):
        e = {0: 7, 7: 300, 300: 301, 301: 900, 900: 1500}[s]
        inc.add(x[s:e])
    assert inc.ntotal == one.ntotal == 1500
    assert bool((inc.lcap >= inc.lsize).all()) and int(inc.lsize.sum()) == 1500
    v0, i0 = one.search(q, 8)
    v1, i1 = inc.search(q, 8)
    assert torch.equal(i0, i1)
    torch.testing.assert_close(v0, v1)
    flat = FlatIndex(16, metric)
    flat.add(x)
    vf, fi = flat.search(q, 8)
    assert torch.equal(i0, fi)
    torch.testing.assert_close(v0, vf, rtol=1e-4, atol=1e-4)


def test_segment_mean_reference():
    from rag_tl_domainllm_optimizer_amd.ops import reference as ref

    g = torch.Generator().manual_seed(0)
    x = torch.randn(50, 8, generator=g)
    a = torch.randint(0, 6, (50,), generator=g)
    a[a == 3] = 2  # one empty cluster
    srt, order = torch.sort(a, stable=True)
    seg = torch.searchsorted(srt, torch.arange(7)).int()
    out = torch.full((6, 8), 7.0)
    ref.segment_mean(x, order, seg, False, out)
    for c in range(6):
        want = x[a == c].mean(0) if (a == c).any() else torch.full((8,), 7.0)
        torch.testing.assert_close(out[c], want)


def test_index_save_load_roundtrip(tmp_path):
    x = _clustered(400, 16)
    q = _clustered(8, 16, seed=9)
    for idx in (FlatIndex(16, "l2"), IVFIndex(16, nlist=8, nprobe=3)):
        if isinstance(idx, IVFIndex):
            idx.train(x, niter=3)
        idx.add(x)
        p = tmp_path / idx.kind
        idx.save(str(p))
        back = load_index(str(p))
        assert type(back) is type(idx) and back.ntotal == idx.ntotal
        v0, i0 = idx.search(q, 4)
        v1, i1 = back.search(q, 4)
        assert torch.equal(i0, i1)
        torch.testing.assert_close(v0, v1)


def test_chunking_windows_and_sources():
    words = [f"w{i}" for i in range(250)]
    ch = chunk_text(" ".join(words), chunk_words=100, overlap=20)
    assert [c.split()[0] for c in ch] == ["w0", "w80", "w160"]
    assert ch[-1].split()[-1] == "w249" and all(len(c.split()) <= 100 for c in ch)
    assert chunk_text("   ") == [] and chunk_text("a b c", 10, 2) == ["a b c"]
    chunks, src = chunk_documents(["x y", " ".join(words)], 100, 20)
    assert src == [0, 1, 1, 1] and chunks[0] == "x y"


def test_encoder_batched_order_independent_and_dedup():
    from rag_tl_domainllm_optimizer_amd.retrieval import Encoder

    enc = Encoder.from_name("tiny-bert", batch_size=3)
    texts = ["alpha beta", "gamma", "alpha beta gamma delta epsilon", "zeta eta", "gamma"]
    e = enc.encode(texts)
    assert e.shape == (5, enc.dim)
    torch.testing.assert_close(e.norm(dim=-1), torch.ones(5), rtol=1e-4, atol=1e-4)
    # a row does not depend on its batch-mates or on padding
    for i, t in enumerate(texts):
        torch.testing.assert_close(enc.encode([t])[0], e[i], rtol=1e-4, atol=1e-5)
    u, where = enc.encode_unique(texts)
    assert u.shape[0] == 4 and where.tolist() == [0, 1, 2, 3, 1]
    torch.testing.assert_close(u[where], e, rtol=1e-4, atol=1e-5)
