"""Vector indexes resident in device memory (HBM on MI355X).

* FlatIndex — exact search: one MFMA GEMM (queries x database, fp32 scores) + radix-select top-k.
* IVFIndex  — inverted file: spherical k-means coarse quantiser (GEMM assignment on device,
  k-means++ seeding and the list build in native host code), vectors stored contiguously per list,
  search = coarse GEMM -> top-nprobe lists -> list-scan kernel -> top-k with id remap.

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
        self.vecs = torch.cat([self.vecs, x.to(self.vecs.dtype)], 0)
        self.ids = torch.cat([self.ids, ids.to(self.device).long()], 0)
        self.sqnorm = torch.cat([self.sqnorm, x.float().pow(2).sum(-1)], 0)
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
    kind = "ivf"

    def __init__(self, dim: int, nlist: int = 256, metric: str = "ip", device="cpu", nprobe: int = 16):
        assert metric in ("ip", "l2")
        self.dim, self.nlist, self.metric, self.nprobe = dim, nlist, metric, nprobe
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.dtype = torch.bfloat16 if self.gpu else torch.float32
        self.centroids = None
        self.vecs = torch.empty(0, dim, dtype=self.dtype, device=self.device)
        self.ids = torch.empty(0, dtype=torch.long, device=self.device)
        self.offsets = torch.zeros(nlist + 1, dtype=torch.int32, device=self.device)
        self.maxlen = 0

    @property
    def ntotal(self) -> int:
        return self.ids.numel()

    @property
    def is_trained(self) -> bool:
        return self.centroids is not None

    # ------------------------------------------------------------------ training
    def _assign(self, x: torch.Tensor, bs: int = 65536) -> torch.Tensor:
        """nearest centroid per row (by the index metric)."""
        out = torch.empty(x.shape[0], dtype=torch.long, device=self.device)
        cen = _pad_rows(self.centroids.to(self.dtype), 128).contiguous() if self.gpu else self.centroids
        cn = self.centroids.float().pow(2).sum(-1)
        for s in range(0, x.shape[0], bs):
            xb = x[s:s + bs].to(self.device)
            if self.gpu:
                sc = ops.gemm(xb.to(self.dtype).contiguous(), cen, out_f32=True)[:, :self.nlist]
            else:
                sc = xb.float() @ self.centroids.float().t()
            if self.metric == "l2":
                sc = 2 * sc - cn[None]
            out[s:s + bs] = sc.argmax(-1)
        return out

    @torch.no_grad()
    def train(self, x: torch.Tensor, niter: int = 20, seed: int = 0, sample: int = 65536):
        from ..ops._ext import native

        x = x.float()
        n = x.shape[0]
        g = torch.Generator(device="cpu").manual_seed(seed)
        if n > sample:
            x = x[torch.randperm(n, generator=g)[:sample].to(x.device)]
        nlist = min(self.nlist, x.shape[0])
        self.nlist = nlist
        self.offsets = torch.zeros(nlist + 1, dtype=torch.int32, device=self.device)
        xs = x.cpu()
        seed_rows = native().kmeanspp_init(xs[: min(len(xs), 16384)], nlist, seed)
        cen = xs[seed_rows].to(self.device)
        xd = x.to(self.device)
        for _ in range(niter):
            self.centroids = cen
            a = self._assign(xd)
            sums = torch.zeros(nlist, self.dim, device=self.device)
            sums.index_add_(0, a, xd)
            cnt = torch.bincount(a, minlength=nlist).float()
            empty = cnt == 0
            cen = sums / cnt.clamp(min=1)[:, None]
            if empty.any():
                ridx = torch.randint(0, xd.shape[0], (int(empty.sum()),), generator=g).to(self.device)
                cen[empty] = xd[ridx]
            if self.metric == "ip":
                cen = torch.nn.functional.normalize(cen, dim=-1)
        self.centroids = cen.float()

    # ------------------------------------------------------------------ add / search
    @torch.no_grad()
    def add(self, x: torch.Tensor, ids: Optional[torch.Tensor] = None):
        from ..ops._ext import native

        assert self.is_trained, "IVFIndex.add before train"
        x = x.to(self.device)
        if ids is None:
            ids = torch.arange(self.ntotal, self.ntotal + x.shape[0], device=self.device)
        # merge with existing content and rebuild lists (counting sort in native host code)
        allx = torch.cat([self.vecs.float(), x.float()], 0) if self.ntotal else x.float()
        allid = torch.cat([self.ids, ids.to(self.device).long()], 0) if self.ntotal else ids.to(self.device).long()
        a = self._assign(allx)
        offsets, order = native().ivf_build_lists(a.cpu(), self.nlist)
        order = order.to(self.device)
        self.vecs = allx[order].to(self.dtype).contiguous()
        self.ids = allid[order].contiguous()
        self.offsets = offsets.to(self.device)
        sizes = offsets[1:] - offsets[:-1]
        self.maxlen = int(sizes.max()) if sizes.numel() else 0

    def search(self, q: torch.Tensor, k: int, nprobe: Optional[int] = None):
        if q.dim() == 1:
            q = q[None]
        nprobe = min(nprobe or self.nprobe, self.nlist)
        q = q.to(self.device)
        nq = q.shape[0]
        # coarse quantiser
        if self.gpu:
            cen = _pad_rows(self.centroids.to(self.dtype), 128).contiguous()
            cs = ops.gemm(q.to(self.dtype).contiguous(), cen, out_f32=True)[:, :self.nlist].contiguous()
        else:
            cs = q.float() @ self.centroids.float().t()
        if self.metric == "l2":
            cs = 2 * cs - self.centroids.float().pow(2).sum(-1)[None]
        probes = torch.topk(cs, nprobe, dim=-1).indices
        if self.gpu and self.metric == "ip" and self.dim % 8 == 0:
            cand, cid = ops.ivf_scan(q.to(self.dtype), probes, self.offsets, self.vecs, self.ids, max(self.maxlen, 1))
            kk = min(k, cand.shape[1])
            v, i = ops.topk(cand, kk)
            ids = cid.gather(1, i.clamp(min=0))
            ids = torch.where(torch.isfinite(v), ids, torch.full_like(ids, -1))
            return v, ids
        # generic path (CPU / l2)
        res_v = torch.full((nq, k), float("-inf"), device=self.device)
        res_i = torch.full((nq, k), -1, dtype=torch.long, device=self.device)
        off = self.offsets.long().cpu()
        for qi in range(nq):
            rows = torch.cat([torch.arange(int(off[l]), int(off[l + 1])) for l in probes[qi].tolist()])
            if rows.numel() == 0:
                continue
            rows = rows.to(self.device)
            xv = self.vecs[rows].float()
            s = xv @ q[qi].float()
            if self.metric == "l2":
                s = 2 * s - xv.pow(2).sum(-1) - q[qi].float().pow(2).sum()
            kk = min(k, s.numel())
            v, i = torch.topk(s, kk)
            res_v[qi, :kk] = v
            res_i[qi, :kk] = self.ids[rows[i]]
        if self.metric == "l2":
            res_v = -res_v
        return res_v, res_i

    # ------------------------------------------------------------------ persistence
    def state(self):
        return {"vecs": self.vecs.float().cpu(), "ids": self.ids.cpu(), "offsets": self.offsets.cpu(),
                "centroids": self.centroids.float().cpu()}, \
               {"kind": self.kind, "dim": self.dim, "metric": self.metric, "nlist": self.nlist, "nprobe": self.nprobe}

    def load_state(self, t):
        self.vecs = t["vecs"].to(self.device, self.dtype)
        self.ids = t["ids"].to(self.device)
        self.offsets = t["offsets"].to(self.device)
        self.centroids = t["centroids"].to(self.device)
        sizes = t["offsets"][1:] - t["offsets"][:-1]
        self.maxlen = int(sizes.max()) if sizes.numel() else 0

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
