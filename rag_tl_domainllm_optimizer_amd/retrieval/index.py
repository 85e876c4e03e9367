"""Vector indexes resident in device memory (HBM on MI355X).

* FlatIndex — exact search: one MFMA GEMM (queries x database, fp32 scores) + radix-select top-k.
* IVFIndex  — inverted file: k-means coarse quantiser trained on device (GEMM + top-1 assignment,
  segmented-mean update kernel; k-means++ seeding in native host code), capacity-padded inverted
  lists with incremental on-device add, search = coarse GEMM -> top-nprobe lists -> list-scan
  kernel (ip or l2) -> top-k with id remap.

A 100k x 384 bf16 database is 77 MB: the whole index lives in HBM next to the models.
Metrics: "ip" (inner product; cosine for normalised vectors) and "l2".
"""
from __future__ import annotations

import json
import os
from typing import Optional, Tuple

import torch

from .. import ops


def _pad_rows(x: torch.Tensor, mult: int) -> torch.Tensor:
    n = x.shape[0]
    m = (n + mult - 1) // mult * mult
    if m == n:
        return x
    return torch.cat([x, torch.zeros(m - n, *x.shape[1:], dtype=x.dtype, device=x.device)], 0)


class FlatIndex:
    kind = "flat"

    def __init__(self, dim: int, metric: str = "ip", device="cpu"):
        assert metric in ("ip", "l2")
        self.dim, self.metric = dim, metric
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.vecs = torch.empty(0, dim, dtype=torch.bfloat16 if self.gpu else torch.float32, device=self.device)
        self.ids = torch.empty(0, dtype=torch.long, device=self.device)
        self.sqnorm = torch.empty(0, dtype=torch.float32, device=self.device)
        self._padded = None

    @property
    def ntotal(self) -> int:
        return self.ids.numel()

    def add(self, x: torch.Tensor, ids: Optional[torch.Tensor] = None):
        x = x.to(self.device)
        if ids is None:
            ids = torch.arange(self.ntotal, self.ntotal + x.shape[0], device=self.device)
        xs = x.to(self.vecs.dtype)
        self.vecs = torch.cat([self.vecs, xs], 0)
        self.ids = torch.cat([self.ids, ids.to(self.device).long()], 0)
        # |x|^2 of the stored (bf16 on GPU) vector: distances are exact w.r.t. what is stored
        self.sqnorm = torch.cat([self.sqnorm, xs.float().pow(2).sum(-1)], 0)
        self._padded = None

    def _db(self):
        if self._padded is None:
            self._padded = _pad_rows(self.vecs, 128).contiguous() if self.gpu else self.vecs
        return self._padded

    def scores(self, q: torch.Tensor) -> torch.Tensor:
        """[nq, ntotal] similarity (higher is better): ip, or -||q-x||^2 for l2."""
        q = q.to(self.device)
        n = self.ntotal
        if self.gpu:
            s = ops.gemm(q.to(torch.bfloat16).contiguous(), self._db(), out_f32=True)[:, :n]
        else:
            s = q.float() @ self.vecs.float().t()
        if self.metric == "l2":
            s = 2 * s - self.sqnorm[None, :] - q.float().pow(2).sum(-1, keepdim=True)
        return s

    def search(self, q: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """-> (scores [nq, k] descending, ids [nq, k]); l2 returns squared distances ascending."""
        if q.dim() == 1:
            q = q[None]
        k = min(k, self.ntotal)
        s = self.scores(q)
        if self.gpu:
            v, i = ops.topk(s.contiguous(), k)
        else:
            v, i = torch.topk(s, k, dim=-1)
        ids = self.ids[i]
        if self.metric == "l2":
            v = -v
        return v, ids

    # ------------------------------------------------------------------ persistence
    def state(self):
        return {"vecs": self.vecs.float().cpu(), "ids": self.ids.cpu(), "sqnorm": self.sqnorm.cpu()}, \
               {"kind": self.kind, "dim": self.dim, "metric": self.metric}

    def load_state(self, t):
        self.vecs = t["vecs"].to(self.device, torch.bfloat16 if self.gpu else torch.float32)
        self.ids = t["ids"].to(self.device)
        self.sqnorm = t["sqnorm"].to(self.device)
        self._padded = None

    def save(self, path: str):
        _save(self, path)


class IVFIndex:
    """Inverted-file index, entirely device-resident on GPU.

    Storage: one bf16 slab ``vecs`` holding every inverted list contiguously with spare capacity
    (``lstart``/``lsize``/``lcap`` per list, int32), the external ``ids`` and the per-slot squared
    norm ``sqnorm`` (for the L2 metric) beside it. ``add`` is incremental: new vectors are assigned
    on device and scattered to the tail of their lists; only when a list overflows are the lists
    re-laid out with 1.5x headroom (amortised O(1) per vector, all on device).

    Training (spherical k-means for "ip", plain k-means for "l2"): k-means++ seeding in native host
    code on a <=16k sample, then per iteration a coarse-quantiser GEMM + fused top-1
    (``ops.gemm`` / ``ops.topk``), a device sort by assignment and the ``segment_mean`` kernel
    (deterministic per-centroid mean, L2-normalised for "ip").

    Search: coarse GEMM -> top-nprobe lists (``ops.topk``) -> ``ivf_scan`` list-scan kernel (ip or
    -||q-x||^2) -> top-k over the candidates. CPU tensors run the same algorithm with torch ops.
    The reference has no vector index at all (README.md:28 declares FAISS/ChromaDB).
    """

    kind = "ivf"

    def __init__(self, dim: int, nlist: int = 256, metric: str = "ip", device="cpu", nprobe: int = 16):
        assert metric in ("ip", "l2")
        self.dim, self.nlist, self.metric, self.nprobe = dim, nlist, metric, nprobe
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.dtype = torch.bfloat16 if self.gpu else torch.float32
        self.centroids = None
        self._reset_lists(nlist)

    def _reset_lists(self, nlist):
        z = lambda: torch.zeros(nlist, dtype=torch.int32, device=self.device)  # noqa: E731
        self.lstart, self.lsize, self.lcap = z(), z(), z()
        self.vecs = torch.empty(0, self.dim, dtype=self.dtype, device=self.device)
        self.ids = torch.empty(0, dtype=torch.long, device=self.device)
        self.sqnorm = torch.empty(0, dtype=torch.float32, device=self.device)
        self.maxlen = 0
        self._ntotal = 0

    @property
    def ntotal(self) -> int:
        return self._ntotal

    @property
    def is_trained(self) -> bool:
        return self.centroids is not None

    @property
    def offsets(self) -> torch.Tensor:
        """Exclusive prefix sum of the list sizes (the compacted layout), int32 [nlist + 1]."""
        z = torch.zeros(1, dtype=torch.int32, device=self.device)
        return torch.cat([z, torch.cumsum(self.lsize, 0).int()])

    # ------------------------------------------------------------------ coarse quantiser
    def _set_centroids(self, cen: torch.Tensor):
        self.centroids = cen.float().contiguous()
        n = self.centroids.shape[0]
        # score(x, c) = x.c - pen[c]: pen = |c|^2 / 2 for l2 (argmax == nearest), 0 for ip;
        # padding rows of the GEMM operand get +inf so they never win
        pen = self.centroids.pow(2).sum(-1) * 0.5 if self.metric == "l2" else torch.zeros(n, device=self.device)
        if self.gpu:
            self._cen_op = _pad_rows(self.centroids.to(self.dtype), 128).contiguous()
            self._pen = torch.full((self._cen_op.shape[0],), float("inf"), device=self.device)
            self._pen[:n] = pen
        else:
            self._cen_op, self._pen = self.centroids, pen

    def _coarse(self, x: torch.Tensor, k: int) -> torch.Tensor:
        """indices [n, k] of the k best centroids per row (x already on device)."""
        if self.gpu:
            s = ops.gemm(x.to(self.dtype).contiguous(), self._cen_op, out_f32=True)
            s.sub_(self._pen)
            return ops.topk(s, k)[1]
        s = x.float() @ self._cen_op.t() - self._pen
        return torch.topk(s, k, dim=-1).indices

    def _assign(self, x: torch.Tensor, bs: int = 65536) -> torch.Tensor:
        """nearest centroid per row (by the index metric), int64 [n]."""
        out = torch.empty(x.shape[0], dtype=torch.long, device=self.device)
        for s in range(0, x.shape[0], bs):
            out[s:s + bs] = self._coarse(x[s:s + bs].to(self.device), 1)[:, 0]
        return out

    # ------------------------------------------------------------------ training
    @torch.no_grad()
    def train(self, x: torch.Tensor, niter: int = 20, seed: int = 0, sample: int = 65536):
        from ..ops._ext import native

        n = x.shape[0]
        g = torch.Generator(device="cpu").manual_seed(seed)
        if n > sample:
            x = x[torch.randperm(n, generator=g)[:sample].to(x.device)]
        nlist = min(self.nlist, x.shape[0])
        self.nlist = nlist
        self._reset_lists(nlist)
        xs = x[: min(len(x), 16384)].float().cpu()
        seed_rows = native().kmeanspp_init(xs, nlist, seed)
        xd = x.to(self.device).float().contiguous()
        xq = xd.to(self.dtype) if self.gpu else xd
        cen = xs[seed_rows].to(self.device)
        if self.metric == "ip":
            cen = torch.nn.functional.normalize(cen, dim=-1)
        grid = torch.arange(nlist + 1, device=self.device)
        for _ in range(niter):
            self._set_centroids(cen)
            a = self._assign(xq)
            srt, order = torch.sort(a, stable=True)
            seg = torch.searchsorted(srt, grid).int()
            new = cen.clone()
            ops.segment_mean(xd, order, seg, self.metric == "ip", new)
            empty = seg[1:] == seg[:-1]
            ne = int(empty.sum())
            if ne:  # reseed empty clusters with random training rows
                ridx = torch.randint(0, xd.shape[0], (ne,), generator=g).to(self.device)
                r = xd[ridx]
                new[empty] = torch.nn.functional.normalize(r, dim=-1) if self.metric == "ip" else r
            cen = new
        self._set_centroids(cen)

    # ------------------------------------------------------------------ add / search
    def _grow(self, need: torch.Tensor):
        """Re-lay the lists out with capacity >= need (1.5x headroom, multiples of 16)."""
        cap = torch.maximum(need, self.lcap + self.lcap // 2)
        cap = ((cap + 15) // 16 * 16).int()
        start = (torch.cumsum(cap, 0) - cap).int()
        total = int(cap.sum())
        vecs = torch.empty(total, self.dim, dtype=self.dtype, device=self.device)
        ids = torch.full((total,), -1, dtype=torch.long, device=self.device)
        sq = torch.zeros(total, dtype=torch.float32, device=self.device)
        if self._ntotal:
            lists = torch.repeat_interleave(torch.arange(self.nlist, device=self.device), self.lsize.long())
            first = (torch.cumsum(self.lsize, 0) - self.lsize).long()
            within = torch.arange(lists.numel(), device=self.device) - first[lists]
            src = self.lstart.long()[lists] + within
            dst = start.long()[lists] + within
            vecs[dst] = self.vecs[src]
            ids[dst] = self.ids[src]
            sq[dst] = self.sqnorm[src]
        self.vecs, self.ids, self.sqnorm = vecs, ids, sq
        self.lstart, self.lcap = start, cap

    @torch.no_grad()
    def add(self, x: torch.Tensor, ids: Optional[torch.Tensor] = None):
        assert self.is_trained, "IVFIndex.add before train"
        n = x.shape[0]
        if n == 0:
            return
        xq = x.to(self.device).to(self.dtype).contiguous()
        ids = (torch.arange(self._ntotal, self._ntotal + n, device=self.device) if ids is None
               else ids.to(self.device).long())
        a = self._assign(xq)
        cnt = torch.bincount(a, minlength=self.nlist).int()
        need = self.lsize + cnt
        if bool((need > self.lcap).any()):
            self._grow(need)
        srt, order = torch.sort(a, stable=True)
        first = (torch.cumsum(cnt, 0) - cnt).long()
        rank = torch.arange(n, device=self.device) - first[srt]
        pos = self.lstart.long()[srt] + self.lsize.long()[srt] + rank
        xs = xq[order]
        self.vecs[pos] = xs
        self.ids[pos] = ids[order]
        self.sqnorm[pos] = xs.float().pow(2).sum(-1)
        self.lsize = need.int()
        self._ntotal += n
        self.maxlen = int(self.lsize.max())

    def search(self, q: torch.Tensor, k: int, nprobe: Optional[int] = None):
        """-> (scores [nq, k] descending (l2: squared distances ascending), ids [nq, k]; -1 pads)."""
        if q.dim() == 1:
            q = q[None]
        nprobe = min(nprobe or self.nprobe, self.nlist)
        q = q.to(self.device)
        l2 = self.metric == "l2"
        probes = self._coarse(q, nprobe)
        maxlen = max(self.maxlen, 1)
        kk = min(k, nprobe * maxlen)
        if self.gpu:
            cand, cid = ops.ivf_scan(q.to(self.dtype), probes, self.lstart, self.lsize, self.vecs, self.ids, maxlen,
                                     self.sqnorm, l2)
            v, i = ops.topk(cand, kk)
        else:
            # same algorithm as the list-scan kernel: [nq, nprobe, maxlen] candidate slots
            j = torch.arange(maxlen)
            slot = self.lstart.long()[probes][..., None] + j
            valid = j < self.lsize.long()[probes][..., None]
            slot = torch.where(valid, slot, torch.zeros_like(slot)).reshape(q.shape[0], -1)
            valid = valid.reshape(q.shape[0], -1)
            xv = self.vecs[slot] if self.vecs.numel() else torch.zeros(*slot.shape, self.dim)
            cand = (xv * q.float()[:, None, :]).sum(-1)
            if l2:
                cand = 2 * cand - self.sqnorm[slot] - q.float().pow(2).sum(-1, keepdim=True)
            cand = torch.where(valid, cand, torch.full_like(cand, float("-inf")))
            cid = torch.where(valid, self.ids[slot] if self.ids.numel() else slot, torch.full_like(slot, -1))
            v, i = torch.topk(cand, kk, dim=-1)
        out_ids = cid.gather(1, i.clamp(min=0))
        out_ids = torch.where(torch.isfinite(v), out_ids, torch.full_like(out_ids, -1))
        if kk < k:
            v = torch.cat([v, torch.full((v.shape[0], k - kk), float("-inf"), device=v.device)], 1)
            out_ids = torch.cat([out_ids, torch.full((v.shape[0], k - kk), -1, dtype=torch.long,
                                                     device=v.device)], 1)
        if l2:
            v = -v
        return v, out_ids

    # ------------------------------------------------------------------ persistence
    def state(self):
        """Compacted lists (no spare capacity) + centroids."""
        lists = torch.repeat_interleave(torch.arange(self.nlist, device=self.device), self.lsize.long())
        first = (torch.cumsum(self.lsize, 0) - self.lsize).long()
        src = self.lstart.long()[lists] + torch.arange(lists.numel(), device=self.device) - first[lists]
        return {"vecs": self.vecs[src].float().cpu(), "ids": self.ids[src].cpu(), "offsets": self.offsets.cpu(),
                "centroids": self.centroids.float().cpu()}, \
               {"kind": self.kind, "dim": self.dim, "metric": self.metric, "nlist": self.nlist, "nprobe": self.nprobe}

    def load_state(self, t):
        off = t["offsets"].to(self.device).int()
        self.nlist = off.numel() - 1
        self._set_centroids(t["centroids"].to(self.device))
        self.lstart = off[:-1].contiguous()
        self.lsize = (off[1:] - off[:-1]).contiguous()
        self.lcap = self.lsize.clone()
        self.vecs = t["vecs"].to(self.device, self.dtype).contiguous()
        self.ids = t["ids"].to(self.device)
        self.sqnorm = self.vecs.float().pow(2).sum(-1)
        self._ntotal = self.ids.numel()
        self.maxlen = int(self.lsize.max()) if self.nlist else 0

    def save(self, path: str):
        _save(self, path)


def _save(index, path: str):
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    tensors, meta = index.state()
    save_file({k: v.contiguous() for k, v in tensors.items()}, os.path.join(path, "index.safetensors"))
    with open(os.path.join(path, "index.json"), "w") as f:
        json.dump(meta, f, indent=2)


def load_index(path: str, device="cpu"):
    from safetensors.torch import load_file

    with open(os.path.join(path, "index.json")) as f:
        meta = json.load(f)
    t = load_file(os.path.join(path, "index.safetensors"))
    if meta["kind"] == "flat":
        idx = FlatIndex(meta["dim"], meta["metric"], device)
    else:
        idx = IVFIndex(meta["dim"], meta["nlist"], meta["metric"], device, meta.get("nprobe", 16))
    idx.load_state(t)
    return idx
