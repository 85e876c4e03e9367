// Attention kernels for gfx950 (SURVEY K4 flash prefill fwd/bwd, K5 decode, K11 encoder attention).
//
// Layout convention: activations are token-major rows ([B*S, ld]) with head h at column h*D, so
// q/k/v are read straight out of the fused qkv projection output and O feeds o_proj directly.
//
// Forward (attn_fwd_kernel<D>): one workgroup = 128 query rows of one (batch, head), 4 waves x 32
// rows. S^T = K·Q^T is computed "swapped" (key on the MFMA row, query on the lane): the S^T
// accumulator of mfma_f32_16x16x32_bf16 is then, after bf16 packing, exactly the A operand of
// P·V (cdna_hip_programming.md §3 'An accumulator tile as the next MFMA's operand'), so P never
// touches LDS; V's B operand comes from ds_read_b64_tr_b16 (T10). K is XOR-swizzled for
// conflict-free ds_read_b128 (T2), V for conflict-free transposed reads. K/V tiles are register-
// prefetched one tile ahead (T14 split: issue before compute, LDS write after the barrier).
// Masks: causal, sliding window, per-batch key start (left padding) and key length (encoder
// padding), plus an optional additive relative-position bias LUT (MPNet).
//
// Decode (attn_decode_kernel + attn_decode_combine_kernel): split-K over the KV cache; one
// workgroup = (partition of keys, kv head, batch) and computes all G = Hq/Hkv query heads that
// share the kv head (the KV cache is read once); per-partition (m, l, o) partials combined by a
// second kernel. Fixed grid sized for the cache capacity -> safe under hipGraph replay with
// device-side lengths.
//
// Backward (attn_bwd_kernel<D>): FA2-style. One workgroup = 64 keys of one (batch, kv head);
// waves own 16 keys each and keep dK^T, dV^T in accumulators while sweeping the group's query
// heads x 64-row query tiles. S and dP are computed with the key on the lane so their
// accumulators are directly the B operands of dV^T = dO^T·P and dK^T = Q^T·dS. dQ is a separate
// kernel (attn_bwd_dq_kernel: query rows per workgroup, no atomics).
#include "rt_common.h"

#include <algorithm>
#include <type_traits>

namespace rt {

typedef __attribute__((address_space(3))) void lds_void;  // global_load_lds destination

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ s16x4 ds_tr16(const void* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
}

__device__ __forceinline__ bf16x8 pack_bf16x8(const f32x4& a, const f32x4& b) {
  uint4 v;
  v.x = pack2bf(a[0], a[1]);
  v.y = pack2bf(a[2], a[3]);
  v.z = pack2bf(b[0], b[1]);
  v.w = pack2bf(b[2], b[3]);
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 cat_tr(s16x4 lo, s16x4 hi) {
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// (x, y, z) of a workgroup after an XCD-aware remap of the linear dispatch id: the workgroups that
// share a K / V head (the query tiles of the G query heads of one kv head, or a kv head's key
// blocks) are consecutive in (x, y, z) order and land on ONE XCD's L2 instead of being dealt round
// robin over all eight (each of which would fetch the K / V / Q tiles from memory again)
//
// lpt != 0 (causal grids, tuning().attn_lpt): the same XCD gets the same set of workgroups, but
// dispatches them heaviest first (longest-processing-time order): a causal tile's work grows with x
// (lpt = 1: query tiles) or shrinks with it (lpt = 2: key blocks of the backward). With ~5
// workgroups per slot and a 1:5 light:heavy spread, x-ascending order leaves the heavy tiles of the
// last groups as the launch's tail. A bijection of the XCD's contiguous range [base, base + cnt):
// dispatch position s walks the x values heaviest first, within one x the groups in order.
__device__ __forceinline__ int3 attn_block_xyz(int lpt = 0) {
  const int nx = gridDim.x, ny = gridDim.y, nwg = nx * ny * gridDim.z;
  const int orig = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
  if (lpt == 0 || nx == 1) {
    const int lin = xcd_remap(orig, nwg);
    return make_int3(lin % nx, (lin / nx) % ny, lin / (nx * ny));
  }
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  const int end = base + (xcd < r ? q + 1 : q);
  int s = orig / 8;  // dispatch position within the XCD
  const int bmod = base % nx;
  for (int i = 0; i < nx; ++i) {
    const int v = lpt == 1 ? nx - 1 - i : i;
    const int first = base + (v - bmod + nx) % nx;  // first lin >= base with lin % nx == v
    const int c = first < end ? (end - 1 - first) / nx + 1 : 0;
    if (s < c) {
      const int lin = first + s * nx;
      return make_int3(v, (lin / nx) % ny, lin / (nx * ny));
    }
    s -= c;
  }
  return make_int3(0, 0, 0);  // not reached: the counts over v sum to the range length
}

struct AttnArgs {
  const bf16_t* q; long ldq;
  const bf16_t* k; long ldk;
  const bf16_t* v; long ldv;
  bf16_t* o; long ldo;
  float* lse;                 // [B, Hq, Sq] (may be null)
  const int* kv_start;        // [B] or null
  const int* kv_len;          // [B] or null
  const float* rel_bias;      // [Hq, 2*rb_L - 1] (log2-domain scaled on host) or null
  int rb_L;
  int B, Sq, Sk, Hq, Hkv;
  int causal, window;
  float scale_log2;           // softmax scale * log2(e)
  int lpt;                    // heaviest-first dispatch order (attn_block_xyz; causal grids)
};

// byte offset of 16-B chunk c of row r in a K-style (row-read) tile image
template <int D>
__device__ __forceinline__ int k_off(int r, int c) {
  constexpr int NCH = D / 8;
  return r * (D * 2) + ((c ^ (r & (NCH - 1))) << 4);
}
// byte offset of 16-B chunk c of row r in a V-style (transposed-read) tile image
template <int D>
__device__ __forceinline__ int v_off(int r, int c) {
  constexpr int NCH = D / 8;
  constexpr int RPB = 128 / D;
  return r * (D * 2) + ((c ^ (((r / RPB) & (NCH / 2 - 1)) << 1)) << 4);
}

// ---------------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------------
// NU = 16-row query blocks per wave: 2 -> 4 waves of 32 rows (256 threads; the launched form), 1 -> 8
// waves of 16 rows (512 threads). Either way a workgroup owns 128 query rows. The occupancy hint
// follows the LDS footprint (D = 128: two 64-KiB double-buffered workgroups per CU), not the wave
// count, so the register cap never forces spills that the LDS would not allow to pay off.
//
// HP (head-packed, GQA with G = 4, NU = 2): a workgroup = 32 query positions x the 4 query heads of
// one kv head (wave w = head 4 hk + w), instead of 128 positions of one head. The 4 waves share
// every K / V tile as before, but all of them have the same causal key range, so short sequences
// (training / reference forwards at S ~ 300) stop spending tiles on rows the diagonal has already
// passed: the 128-row tile's waves ran every key tile up to the tile's LAST row. Per row the same
// key tiles in the same order with the same arithmetic (trailing fully masked tiles change
// nothing: alpha = 1, p = 0), so the output and lse are bitwise the 128-row form's.
//
// Q64 (NU = 1, 4 waves of 16 rows): 64 positions of one head per workgroup — the same causal
// saving for heads that share no K / V (MHA, e.g. Llama-2-13B), bitwise the 128-row form too.
template <int D, int NU = 2, bool HP = false, bool Q64 = false>
__global__ __launch_bounds__(Q64 ? 256 : 64 * 8 / NU, D == 128 ? 2 : (D == 64 ? 3 : 4))
void attn_fwd_kernel(AttnArgs a) {
  static_assert(!HP || NU == 2, "HP: 4 waves of 32 rows");
  static_assert(!Q64 || (NU == 1 && !HP), "Q64: 4 waves of 16 rows");
  constexpr int NT = Q64 ? 256 : 64 * 8 / NU;  // threads per workgroup
  constexpr int NCH = D / 8, DS = D / 32, DT = D / 16;
  constexpr int TILE_BYTES = 64 * D * 2;
  constexpr int OROW = D + 8;  // O staging row stride (elements)
  // D >= 64: two K / V tile buffers — the next tile is stored into the other buffer right after the
  // current one is consumed, so each tile costs one barrier (64 KiB per workgroup at D = 128: 2 per
  // CU). D = 32 (4 workgroups per CU, 128 registers) keeps one buffer and two barriers.
  constexpr bool DB = D >= 64;
  constexpr int NBUF = DB ? 2 : 1;
  constexpr int SMEM = (2 * NBUF * TILE_BYTES > 128 * OROW * 2) ? 2 * NBUF * TILE_BYTES : 128 * OROW * 2;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int3 bx = attn_block_xyz(a.lpt);
  const int b = bx.z;
  const int h = HP ? bx.y * 4 + wid : bx.y;
  const int hk = HP ? bx.y : h / (a.Hq / a.Hkv);
  constexpr int QROWS = HP ? 32 : (Q64 ? 64 : 128);  // query positions per workgroup
  const int qblk0 = bx.x * QROWS;
  const int q0 = HP ? qblk0 : qblk0 + wid * 16 * NU;

  const int start = a.kv_start ? a.kv_start[b] : 0;
  int kend = a.kv_len ? min(a.kv_len[b], a.Sk) : a.Sk;
  const int qlast = min(qblk0 + QROWS - 1, a.Sq - 1);
  if (a.causal) kend = min(kend, qlast + 1);
  int kbeg = start;
  if (a.window > 0) kbeg = max(kbeg, qblk0 - a.window + 1);
  kbeg = max(kbeg, 0) & ~63;

  // Q fragments (B operand of S^T = K·Q^T): lane holds Q[q0+16u+r16][32s + 8g .. +8]
  bf16x8 qf[NU][DS];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int qrow = min(q0 + 16 * u + r16, a.Sq - 1);
    const bf16_t* qp = a.q + ((long)b * a.Sq + qrow) * a.ldq + (long)h * D + 8 * g;
#pragma unroll
    for (int s = 0; s < DS; ++s) qf[u][s] = *(const bf16x8*)(qp + 32 * s);
  }
  // retire the Q loads here, once: otherwise hipcc's wait tracking loses them at the loop header
  // and drains vmcnt(0) before the first S MFMA of EVERY tile — which also waits out the next
  // tile's prefetch and serialises load latency with compute
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int s = 0; s < DS; ++s) asm volatile("" : "+v"(qf[u][s]));

  f32x4 o[NU][DT];
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int c = 0; c < DT; ++c) o[u][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[NU], l[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) { m[u] = -INFINITY; l[u] = 0.f; }

  // register prefetch of one K/V tile: 64 rows x NCH chunks each, spread over 256 threads. Thread
  // tid always owns chunk c = tid % NCH of keys tid / NCH + (256 / NCH) r. Native vector registers
  // (an array of the HIP uint4 struct went to scratch, serialising every prefetch load)
  constexpr int CPT = 64 * NCH / NT;  // chunks per thread per tensor (4 for D=128, 256 threads)
  constexpr int KSTEP = NT / NCH;     // key stride between a thread's chunks
  const int lc = tid % NCH, lkey = tid / NCH;
  const bf16_t* kb = a.k + (long)b * a.Sk * a.ldk + (long)hk * D + lc * 8;
  const bf16_t* vb = a.v + (long)b * a.Sk * a.ldv + (long)hk * D + lc * 8;
  u32x4 kreg[CPT], vreg[CPT];
  auto load_tile = [&](int kv0) {
#pragma unroll
    for (int r = 0; r < CPT; ++r) {
      const long kk = min(kv0 + lkey + KSTEP * r, a.Sk - 1);
      kreg[r] = *(const u32x4*)(kb + kk * a.ldk);
      vreg[r] = *(const u32x4*)(vb + kk * a.ldv);
    }
  };
  auto store_tile = [&](char* kd, char* vd) {
#pragma unroll
    for (int r = 0; r < CPT; ++r) {
      *(u32x4*)(kd + k_off<D>(lkey + KSTEP * r, lc)) = kreg[r];
      *(u32x4*)(vd + v_off<D>(lkey + KSTEP * r, lc)) = vreg[r];
    }
  };

  if (kbeg < kend) {
    load_tile(kbeg);
    store_tile(smem, smem + TILE_BYTES);
  }
  __syncthreads();

  int cur = 0;  // K / V buffer of the tile being consumed (always 0 without double buffering)
  for (int kv0 = kbeg; kv0 < kend; kv0 += 64) {
    const bool has_next = kv0 + 64 < kend;
    if (has_next) load_tile(kv0 + 64);
    char* Ks = DB ? smem + cur * (2 * TILE_BYTES) : smem;
    char* Vs = DB ? Ks + TILE_BYTES : smem + TILE_BYTES;

    // ---- S^T[t][u] = K[16t..][:] · Q[u]^T ----
    f32x4 st[4][NU];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int u = 0; u < NU; ++u) st[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int s = 0; s < DS; ++s) {
        const bf16x8 kf = *(const bf16x8*)(Ks + k_off<D>(16 * t + r16, 4 * s + g));
#pragma unroll
        for (int u = 0; u < NU; ++u) st[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[u][s], st[t][u], 0, 0, 0);
      }

    // ---- scale + mask ----
    const bool full = kv0 >= start && kv0 + 63 < kend && (!a.causal || kv0 + 63 <= q0) &&
                      (a.window <= 0 || (q0 + 16 * NU - 1) - kv0 < a.window) && !a.rel_bias;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float x = st[t][u][i] * a.scale_log2;
          if (!full) {
            const int kk = kv0 + 16 * t + 4 * g + i;
            const int qq = q0 + 16 * u + r16;
            bool ok = kk >= start && kk < kend;
            if (a.causal) ok = ok && kk <= qq;
            if (a.window > 0) ok = ok && (qq - kk) < a.window;
            ok = ok && qq < a.Sq;
            if (a.rel_bias && ok) x += a.rel_bias[(long)h * (2 * a.rb_L - 1) + (kk - qq) + a.rb_L - 1];
            x = ok ? x : -INFINITY;
          }
          st[t][u][i] = x;
        }

    // ---- online softmax (per q column = lane r16 of each u) ----
    float alpha[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) mx = fmaxf(mx, st[t][u][i]);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m[u], mx);
      const float mu = mn == -INFINITY ? 0.f : mn;
      alpha[u] = exp2f(m[u] - mu);
      m[u] = mn;
      float rs = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float pv = exp2f(st[t][u][i] - mu);
          st[t][u][i] = pv;
          rs += pv;
        }
      rs += __shfl_xor(rs, 16, 64);
      rs += __shfl_xor(rs, 32, 64);
      l[u] = l[u] * alpha[u] + rs;
    }
    // rescale O rows (row q = 16u + 4g + i lives in lane 4g+i's alpha)
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float al = __shfl(alpha[u], 4 * g + i, 64);
#pragma unroll
        for (int c = 0; c < DT; ++c) o[u][c][i] *= al;
      }

    // ---- O += P · V ----
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 pa[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) pa[u] = pack_bf16x8(st[2 * ks][u], st[2 * ks + 1][u]);
      const int qrow = lane >> 2 & 3, pcol = lane & 3;  // tr-read addressing within the 16-lane group
#pragma unroll
      for (int c = 0; c < DT; ++c) {
        const int key_a = 32 * ks + 4 * g + qrow;
        const int col = 16 * c + 4 * pcol;  // element column
        const s16x4 lo = ds_tr16(Vs + v_off<D>(key_a, col >> 3) + ((col & 7) << 1));
        const s16x4 hi = ds_tr16(Vs + v_off<D>(key_a + 16, col >> 3) + ((col & 7) << 1));
        const bf16x8 vf = cat_tr(lo, hi);
#pragma unroll
        for (int u = 0; u < NU; ++u) o[u][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[u], vf, o[u][c], 0, 0, 0);
      }
    }
    if constexpr (DB) {
      // the other buffer was last read in the previous iteration, which every wave has left (its
      // closing barrier): store the next tile there and swap
      char* kn = smem + (cur ^ 1) * (2 * TILE_BYTES);
      if (has_next) store_tile(kn, kn + TILE_BYTES);
      __syncthreads();
      cur ^= 1;
    } else {
      __syncthreads();
      if (has_next) store_tile(Ks, Vs);
      __syncthreads();
    }
  }

  // ---- finalize ----
  if (a.lse && g == 0) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int qq = q0 + 16 * u + r16;
      if (qq < a.Sq) {
        const float v = l[u] > 0.f ? (m[u] + __log2f(l[u])) * 0.69314718055994531f : INFINITY;
        a.lse[((long)b * a.Hq + h) * a.Sq + qq] = v;
      }
    }
  }
  bf16_t* Os = (bf16_t*)smem;  // [128][OROW]
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float lr = __shfl(l[u], 4 * g + i, 64);
      const float inv = lr > 0.f ? 1.f / lr : 0.f;
      const int row = wid * 16 * NU + 16 * u + 4 * g + i;
#pragma unroll
      for (int c = 0; c < DT; ++c) Os[row * OROW + 16 * c + r16] = f2bf(o[u][c][i] * inv);
    }
  __syncthreads();
  for (int e = tid; e < (Q64 ? 64 : 128) * NCH; e += NT) {
    const int row = e / NCH, c = e % NCH;
    // HP: staging row 32 w + r = position qblk0 + r of head 4 hk + w
    const int qq = HP ? qblk0 + (row & 31) : qblk0 + row;
    const int hh = HP ? hk * 4 + (row >> 5) : h;
    if (qq < a.Sq)
      *(uint4*)(a.o + ((long)b * a.Sq + qq) * a.ldo + (long)hh * D + c * 8) = *(const uint4*)(Os + row * OROW + c * 8);
  }
}

// ---------------------------------------------------------------------------------------------
// decode (one query token per sequence, KV cache [B, Hkv, Smax, D])
// ---------------------------------------------------------------------------------------------
struct DecodeArgs {
  const bf16_t* q; long ldq;        // [B, ldq], head h at h*D
  const bf16_t* kc; const bf16_t* vc;
  int Smax;
  const int* kv_len;                // [B] valid keys (incl. current token)
  const int* kv_start;              // [B] or null
  int window;
  float* part;                      // [B, Hkv, NP, G, D+2]
  bf16_t* o; long ldo;
  int B, Hq, Hkv, NP, PS;
  float scale_log2;
};

template <int D, int G>
__global__ __launch_bounds__(256) void attn_decode_kernel(DecodeArgs a) {
  constexpr int LPK = D / 8;       // lanes per key (8 d each)
  constexpr int KPW = 64 / LPK;    // keys per wave-step
  extern __shared__ __attribute__((aligned(16))) float dsm[];  // scores [G][PS] + reduce
  float* sc = dsm;
  float* red = dsm + G * a.PS;     // [4 waves][G][D]
  __shared__ float wstat[4][G][2];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int part = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int len = a.kv_len[b];
  int kbeg = a.kv_start ? a.kv_start[b] : 0;
  if (a.window > 0) kbeg = max(kbeg, len - a.window);
  const int p0 = max(part * a.PS, kbeg), p1 = min((part + 1) * a.PS, len);
  float* outp = a.part + ((((long)b * a.Hkv + hk) * a.NP + part) * G) * (D + 2);
  if (p0 >= p1) {
    if (tid < G) { outp[tid * (D + 2) + D] = -INFINITY; outp[tid * (D + 2) + D + 1] = 0.f; }
    return;
  }
  const int sub = lane / LPK, dl = lane % LPK;
  float qv[G][8];
#pragma unroll
  for (int gg = 0; gg < G; ++gg) unpack8(*(const uint4*)(a.q + (long)b * a.ldq + (long)(hk * G + gg) * D + dl * 8), qv[gg]);

  const bf16_t* kbase = a.kc + ((long)b * a.Hkv + hk) * a.Smax * D;
  const bf16_t* vbase = a.vc + ((long)b * a.Hkv + hk) * a.Smax * D;
  // pass 1: scores
  float wmax[G];
#pragma unroll
  for (int gg = 0; gg < G; ++gg) wmax[gg] = -INFINITY;
  for (int key = p0 + wid * KPW + sub; key - sub < p1; key += 4 * KPW) {
    float kv[8];
    const int kk = min(key, p1 - 1);
    unpack8(*(const uint4*)(kbase + (long)kk * D + dl * 8), kv);
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) s += qv[gg][e] * kv[e];
#pragma unroll
      for (int off = LPK / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
      s *= a.scale_log2;
      if (key < p1) {
        if (dl == 0) sc[gg * a.PS + (key - p0)] = s;
        wmax[gg] = fmaxf(wmax[gg], s);
      }
    }
  }
#pragma unroll
  for (int gg = 0; gg < G; ++gg) {
    const float mx = wave_max(wmax[gg]);
    if (lane == 0) wstat[wid][gg][0] = mx;
  }
  __syncthreads();
  float mrow[G];
#pragma unroll
  for (int gg = 0; gg < G; ++gg)
    mrow[gg] = fmaxf(fmaxf(wstat[0][gg][0], wstat[1][gg][0]), fmaxf(wstat[2][gg][0], wstat[3][gg][0]));
  // pass 2: p = exp2(s - m), o += p v
  float acc[G][8], lsum[G];
#pragma unroll
  for (int gg = 0; gg < G; ++gg) {
    lsum[gg] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[gg][e] = 0.f;
  }
  for (int key = p0 + wid * KPW + sub; key - sub < p1; key += 4 * KPW) {
    if (key < p1) {
      float vv[8];
      unpack8(*(const uint4*)(vbase + (long)key * D + dl * 8), vv);
#pragma unroll
      for (int gg = 0; gg < G; ++gg) {
        const float p = exp2f(sc[gg * a.PS + (key - p0)] - mrow[gg]);
        lsum[gg] += p;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[gg][e] += p * vv[e];
      }
    }
  }
  // reduce over the KPW key sub-groups of the wave
#pragma unroll
  for (int gg = 0; gg < G; ++gg) {
#pragma unroll
    for (int off = LPK; off < 64; off <<= 1) {
      lsum[gg] += __shfl_xor(lsum[gg], off, 64);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[gg][e] += __shfl_xor(acc[gg][e], off, 64);
    }
  }
  if (sub == 0) {
#pragma unroll
    for (int gg = 0; gg < G; ++gg)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[(wid * G + gg) * D + dl * 8 + e] = acc[gg][e];
  }
  if (lane == 0)
#pragma unroll
    for (int gg = 0; gg < G; ++gg) wstat[wid][gg][1] = lsum[gg];
  __syncthreads();
  for (int e = tid; e < G * D; e += 256) {
    const int gg = e / D, d = e % D;
    outp[gg * (D + 2) + d] = red[(0 * G + gg) * D + d] + red[(1 * G + gg) * D + d] + red[(2 * G + gg) * D + d] +
                             red[(3 * G + gg) * D + d];
  }
  if (tid < G) {
    outp[tid * (D + 2) + D] = mrow[tid];
    outp[tid * (D + 2) + D + 1] = wstat[0][tid][1] + wstat[1][tid][1] + wstat[2][tid][1] + wstat[3][tid][1];
  }
}

template <int D, int G>
__global__ __launch_bounds__(256) void attn_decode_combine_kernel(DecodeArgs a) {
  // one workgroup per (b, hk); threads over G*D outputs
  const int hk = blockIdx.x, b = blockIdx.y;
  const float* pp = a.part + (((long)b * a.Hkv + hk) * a.NP) * G * (D + 2);
  for (int e = threadIdx.x; e < G * D; e += blockDim.x) {
    const int gg = e / D, d = e % D;
    float M = -INFINITY;
    for (int p = 0; p < a.NP; ++p) M = fmaxf(M, pp[(p * G + gg) * (D + 2) + D]);
    float L = 0.f, O = 0.f;
    if (M != -INFINITY) {
      for (int p = 0; p < a.NP; ++p) {
        const float* q = pp + (p * G + gg) * (D + 2);
        if (q[D] == -INFINITY) continue;  // empty partition: its o[] was never written
        const float w = exp2f(q[D] - M);
        L += w * q[D + 1];
        O += w * q[d];
      }
    }
    a.o[(long)b * a.ldo + (long)(hk * G + gg) * D + d] = f2bf(L > 0.f ? O / L : 0.f);
  }
}

// ---------------------------------------------------------------------------------------------
// Fused decode step: RoPE(q, k_new) + KV-cache append + split-K attention + in-launch combine
// ---------------------------------------------------------------------------------------------
// Replaces rope_qkv + attn_decode + attn_decode_combine (three launches, each a dependent global
// round trip at decode sizes) by one. Grid (NP partitions, Hkv, B); partition p owns keys
// [p*PS, (p+1)*PS). Every lane issues ALL of its K and V loads for the partition up front (NK keys
// each, 16 B per key per operand), so a block costs one memory round trip. The block owning the
// new token's slot rotates k_new, writes k/v into the cache and uses them from registers. Partials
// (m, l, o) go to a workspace; the last-arriving partition of (b, kv-head) merges them (agent-scope
// release -> relaxed ticket -> acquire, as in gemm_decode_kernel) and re-arms the ticket for the
// next graph replay.
struct DecodeFusedArgs {
  const bf16_t* qkv; long ldq;      // [B, ldq] = q heads | k heads | v heads of the new token (pre-RoPE)
  bf16_t* kc; bf16_t* vc; int Smax; // [B, Hkv, Smax, D]
  const int* slot;                  // [B] cache slot of the new token
  const int* attn_len;              // [B] keys attended (normally slot + 1)
  const int* kv_start;              // [B] first valid slot (left padding) or null
  const int* pos;                   // [B] rotary position of the new token
  const float* cosT; const float* sinT; float sign;  // [P, D/2] tables or null (no rotary)
  int window;
  float* part;                      // [B, Hkv, NP, G, D + 2]
  unsigned* tickets;                // [B * Hkv], zero between launches
  bf16_t* o; long ldo;
  int B, Hq, Hkv, NP, PS;
  float scale_log2;
  // optional: qkv as nsplit fp32 split-K slabs [nsplit][B][ldq] (the qkv GEMM's reduce fused into
  // the MFMA kernel's prologue); qkv above is then unused
  const float* qkv_slabs; int qkv_nsplit; long qkv_sstride;
  int kv_nt;                        // MFMA kernel: non-temporal K/V cache loads (each read once per step)
  long long* stamps;                // debug (W > 1 kernel): [blocks * W][8] s_memrealtime phase stamps, or null
  // fp8 K/V cache (config 5, MFMA kernels only): kc / vc hold OCP e4m3fn bytes, one fp32 scale per
  // (batch, kv head, slot) in ksc / vsc [B, Hkv, SmaxP]; K rows are stored k-permuted (element
  // 32 s + 8 g + e at byte 32 g + 8 s + e: one lane's four MFMA K chunks are 32 contiguous bytes)
  float* ksc; float* vsc; int SmaxP;
};

template <int D>
__device__ __forceinline__ void rope_chunk(const bf16_t* head, int dl, const DecodeFusedArgs& a, int p,
                                           float (&out)[8]) {
  constexpr int HALF = D / 16;  // chunks of 8 in half a head
  float x[8];
  unpack8(*(const uint4*)(head + dl * 8), x);
  if (a.cosT) {
    float y[8];
    unpack8(*(const uint4*)(head + (dl ^ HALF) * 8), y);
    const int j0 = (dl & (HALF - 1)) * 8;
    const float* cr = a.cosT + (long)p * (D / 2) + j0;
    const float* sr = a.sinT + (long)p * (D / 2) + j0;
    const float4 c0 = *(const float4*)cr, c1 = *(const float4*)(cr + 4);
    const float4 s0 = *(const float4*)sr, s1 = *(const float4*)(sr + 4);
    const float cs[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const bool lo = dl < HALF;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float sv = a.sign * sn[k];
      // explicit fma order shared by every RoPE site (rope_qkv_kernel): bitwise-equal appends
      out[k] = fmaf(x[k], cs[k], lo ? -(y[k] * sv) : y[k] * sv);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = x[k];
  }
  // the unfused path stores rotated rows in bf16: round identically
#pragma unroll
  for (int k = 0; k < 8; ++k) out[k] = bf2f(f2bf(out[k]));
}

// One key chunk: CH = 4 waves x KPW keys x NK keys per lane. Loads of chunk j+1 are issued before
// chunk j is consumed (two named register sets), softmax is online across chunks.
template <int D, int NK>
struct KVChunk {
  uint4 k[NK], v[NK];
};

template <int D, int NK>
__device__ __forceinline__ void load_chunk(KVChunk<D, NK>& c, const bf16_t* kbase, const bf16_t* vbase, int c0,
                                           int p1, int wid, int sub, int dl, bool nt) {
  constexpr int KPW = 64 / (D / 8);
  if (nt) {
#pragma unroll
    for (int i = 0; i < NK; ++i) {
      const int key = min(c0 + (i * 4 + wid) * KPW + sub, p1 - 1);
      c.k[i] = load_nt16(kbase + (long)key * D + dl * 8);
      c.v[i] = load_nt16(vbase + (long)key * D + dl * 8);
    }
  } else {
#pragma unroll
    for (int i = 0; i < NK; ++i) {
      const int key = min(c0 + (i * 4 + wid) * KPW + sub, p1 - 1);
      c.k[i] = *(const uint4*)(kbase + (long)key * D + dl * 8);
      c.v[i] = *(const uint4*)(vbase + (long)key * D + dl * 8);
    }
  }
}

template <int D, int G, int NK>
__device__ __forceinline__ void consume_chunk(KVChunk<D, NK>& c, int c0, int p1, int s_new, bool has_new,
                                              const uint4& kp, const uint4& vp, const float (&qv)[G][8],
                                              float (&m)[G], float (&l)[G], float (&acc)[G][8], int wid, int sub,
                                              float scale_log2) {
  constexpr int LPK = D / 8, KPW = 64 / LPK;
  if (has_new) {
    // compare the CLAMPED index load_chunk read: lanes past p1 re-read slot p1 - 1, which in a
    // decode step is s_new itself — a slot this very launch is still writing (stale or
    // uninitialised cache memory; masked, but 0 * NaN would poison the PV sum)
#pragma unroll
    for (int i = 0; i < NK; ++i)
      if (min(c0 + (i * 4 + wid) * KPW + sub, p1 - 1) == s_new) { c.k[i] = kp; c.v[i] = vp; }
  }
  float sc[G][NK];
#pragma unroll
  for (int i = 0; i < NK; ++i) {
    float kf[8];
    unpack8(c.k[i], kf);
    const bool ok = c0 + (i * 4 + wid) * KPW + sub < p1;
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      float sdot = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) sdot += qv[gg][e] * kf[e];
#pragma unroll
      for (int off = LPK / 2; off > 0; off >>= 1) sdot += __shfl_xor(sdot, off, 64);
      sc[gg][i] = ok ? sdot * scale_log2 : -INFINITY;
    }
  }
  // per-lane online softmax over this lane's keys (cross-lane merge happens once at the end)
#pragma unroll
  for (int gg = 0; gg < G; ++gg) {
    float cm = sc[gg][0];
#pragma unroll
    for (int i = 1; i < NK; ++i) cm = fmaxf(cm, sc[gg][i]);
    const float mn = fmaxf(m[gg], cm);
    if (mn == -INFINITY) continue;  // nothing valid yet for this lane
    const float r = exp2f(m[gg] - mn);
    l[gg] *= r;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[gg][e] *= r;
    m[gg] = mn;
  }
#pragma unroll
  for (int i = 0; i < NK; ++i) {
    float vf[8];
    unpack8(c.v[i], vf);
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      // masked key -> 0 (also when every key so far was masked: m = -inf would give NaN)
      const float pr = sc[gg][i] == -INFINITY ? 0.f : exp2f(sc[gg][i] - m[gg]);
      l[gg] += pr;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[gg][e] += pr * vf[e];
    }
  }
}

template <int D, int G, int NK>
__global__ __launch_bounds__(256) void attn_decode_fused_kernel(DecodeFusedArgs a) {
  constexpr int LPK = D / 8;    // lanes per key
  constexpr int KPW = 64 / LPK; // keys per wave-step
  constexpr int CH = 4 * KPW * NK;
  __shared__ float red[4 * G * D];
  __shared__ float wst[4][G][2];
  __shared__ int flag;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int part = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int len = a.attn_len[b];
  const int s_new = a.slot[b];
  RT_ASSERT(len <= a.Smax && s_new >= 0 && s_new < a.Smax);
  int kbeg = a.kv_start ? a.kv_start[b] : 0;
  if (a.window > 0) kbeg = max(kbeg, len - a.window);
  const int p0 = max(part * a.PS, kbeg), p1 = min((part + 1) * a.PS, len);
  const int sub = lane / LPK, dl = lane % LPK;
  const bf16_t* row = a.qkv + (long)b * a.ldq;

  float mrow[G], lrow[G];
  const bool active = p0 < p1;
  if (active) {
    const int p = a.pos ? a.pos[b] : 0;
    const bf16_t* kbase = a.kc + ((long)b * a.Hkv + hk) * a.Smax * D;
    const bf16_t* vbase = a.vc + ((long)b * a.Hkv + hk) * a.Smax * D;
    KVChunk<D, NK> ca, cb;
    load_chunk<D, NK>(ca, kbase, vbase, p0, p1, wid, sub, dl, a.kv_nt);
    // the second chunk is issued with the first, before q (waiting for q drains both): a
    // partition of <= 2 chunks (the batch-1 partition plan) costs one memory round trip, not two
    if (p0 + CH < p1) load_chunk<D, NK>(cb, kbase, vbase, p0 + CH, p1, wid, sub, dl, a.kv_nt);
    float qv[G][8];
#pragma unroll
    for (int gg = 0; gg < G; ++gg) rope_chunk<D>(row + (long)(hk * G + gg) * D, dl, a, p, qv[gg]);
    const bool has_new = s_new >= p0 && s_new < p1;
    uint4 kp = make_uint4(0, 0, 0, 0), vp = kp;
    if (has_new) {
      float kn[8], vn[8];
      rope_chunk<D>(row + (long)(a.Hq + hk) * D, dl, a, p, kn);
      unpack8(*(const uint4*)(row + (long)(a.Hq + a.Hkv + hk) * D + dl * 8), vn);
      kp = pack8(kn);
      vp = pack8(vn);
      if (wid == 0 && sub == 0) {
        *(uint4*)(a.kc + (((long)b * a.Hkv + hk) * a.Smax + s_new) * D + dl * 8) = kp;
        *(uint4*)(a.vc + (((long)b * a.Hkv + hk) * a.Smax + s_new) * D + dl * 8) = vp;
      }
    }
    float m[G], l[G], acc[G][8];
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      m[gg] = -INFINITY;
      l[gg] = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[gg][e] = 0.f;
    }
    for (int c0 = p0; c0 < p1; c0 += 2 * CH) {
      if (c0 != p0 && c0 + CH < p1) load_chunk<D, NK>(cb, kbase, vbase, c0 + CH, p1, wid, sub, dl, a.kv_nt);
      consume_chunk<D, G, NK>(ca, c0, p1, s_new, has_new, kp, vp, qv, m, l, acc, wid, sub, a.scale_log2);
      if (c0 + CH < p1) {
        if (c0 + 2 * CH < p1) load_chunk<D, NK>(ca, kbase, vbase, c0 + 2 * CH, p1, wid, sub, dl, a.kv_nt);
        consume_chunk<D, G, NK>(cb, c0 + CH, p1, s_new, has_new, kp, vp, qv, m, l, acc, wid, sub, a.scale_log2);
      }
    }
    // merge lanes holding the same d (different keys): over sub within the wave, then over waves
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      float mw = m[gg];
#pragma unroll
      for (int off = LPK; off < 64; off <<= 1) mw = fmaxf(mw, __shfl_xor(mw, off, 64));
      const float r = (m[gg] == -INFINITY) ? 0.f : exp2f(m[gg] - mw);
      l[gg] *= r;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[gg][e] *= r;
      m[gg] = mw;
      if (lane == 0) wst[wid][gg][0] = mw;
    }
    __syncthreads();
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      mrow[gg] = fmaxf(fmaxf(wst[0][gg][0], wst[1][gg][0]), fmaxf(wst[2][gg][0], wst[3][gg][0]));
      const float r = (m[gg] == -INFINITY) ? 0.f : exp2f(m[gg] - mrow[gg]);
      float lsum = l[gg] * r;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[gg][e] *= r;
#pragma unroll
      for (int off = LPK; off < 64; off <<= 1) {
        lsum += __shfl_xor(lsum, off, 64);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[gg][e] += __shfl_xor(acc[gg][e], off, 64);
      }
      if (sub == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) red[(wid * G + gg) * D + dl * 8 + e] = acc[gg][e];
      }
      if (lane == 0) wst[wid][gg][1] = lsum;
    }
    __syncthreads();
#pragma unroll
    for (int gg = 0; gg < G; ++gg) lrow[gg] = wst[0][gg][1] + wst[1][gg][1] + wst[2][gg][1] + wst[3][gg][1];
  }

  if (a.NP == 1) {
    for (int e = tid; e < G * D; e += 256) {
      const int gg = e / D, d = e % D;
      float ov = 0.f;
      if (active && lrow[gg] > 0.f)
        ov = (red[(0 * G + gg) * D + d] + red[(1 * G + gg) * D + d] + red[(2 * G + gg) * D + d] +
              red[(3 * G + gg) * D + d]) / lrow[gg];
      a.o[(long)b * a.ldo + (long)(hk * G + gg) * D + d] = f2bf(ov);
    }
    return;
  }

  // ---- publish the partial with write-through (agent-scope) stores, take a ticket; the last
  // partition of (b, hk) merges with agent-scope loads. No L2 writeback / invalidate fences:
  // cdna_hip_programming.md / MI355X_MICROARCH.md 'handoff-flag' (drained sc1 payload -> flag).
  float* pp = a.part + (((long)b * a.Hkv + hk) * a.NP) * G * (D + 2);
  float* outp = pp + (long)part * G * (D + 2);
  for (int e = tid; e < G * D; e += 256) {
    const int gg = e / D, d = e % D;
    if (active)
      __hip_atomic_store(outp + gg * (D + 2) + d,
                         red[(0 * G + gg) * D + d] + red[(1 * G + gg) * D + d] + red[(2 * G + gg) * D + d] +
                             red[(3 * G + gg) * D + d],
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid < G) {
    __hip_atomic_store(outp + tid * (D + 2) + D, active ? mrow[tid] : -INFINITY, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(outp + tid * (D + 2) + D + 1, active ? lrow[tid] : 0.f, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(a.tickets + (long)b * a.Hkv + hk, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    flag = (old == (unsigned)(a.NP - 1));
  }
  __syncthreads();
  if (!flag) return;
  for (int e = tid; e < G * D; e += 256) {
    const int gg = e / D, d = e % D;
    float M = -INFINITY, L = 0.f, O = 0.f;
#pragma unroll 4
    for (int q = 0; q < a.NP; ++q) {
      const float* r = pp + (q * G + gg) * (D + 2);
      const float mq = __hip_atomic_load(r + D, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const float lq = __hip_atomic_load(r + D + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const float oq = __hip_atomic_load(r + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (mq == -INFINITY) continue;  // empty partition: o[] never written
      const float Mn = fmaxf(M, mq);
      const float r0 = exp2f(M - Mn), r1 = exp2f(mq - Mn);
      L = L * r0 + lq * r1;
      O = O * r0 + oq * r1;
      M = Mn;
    }
    a.o[(long)b * a.ldo + (long)(hk * G + gg) * D + d] = f2bf(L > 0.f ? O / L : 0.f);
  }
  if (tid == 0) __hip_atomic_store(a.tickets + (long)b * a.Hkv + hk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------------------------
// fp8-cache decode step for MHA (G = 1: Llama-2-13B, config 5) on the VALU
// ---------------------------------------------------------------------------------------------
// With one query head per kv head the MFMA form above computes 16 query rows of which 15 are
// empty, and its fp8 variant moves only 3.6 TB/s (profiles/r3/dec13b_b64_fp8kv_kernels.txt).
// Here one wave owns one (batch, head) and walks 16-key tiles, four in flight:
//   * QK: lane (g, r) dots key c0 + r over elements {32 s + 8 g + e} — the 32 contiguous bytes of
//     the k-permuted fp8 row at byte 32 g — against its 32 q values (fp32 registers, pre-scaled
//     by softmax scale * log2 e); the 4 lane groups' partials meet by two shuffles;
//   * online softmax over the tile's 16 scores (lanes r: 4 shuffles each for max and sum);
//   * PV: lane (g, r) accumulates dims [8 r, 8 r + 8) over keys c0 + 4 i + g (i < 4): 8 V bytes per
//     key, P (with the key's V scale folded in) broadcast from lane 4 i + g.
// The 4 groups' O partials meet once, after the last tile. No LDS and no MFMA. The new token is
// rotated, quantised and appended as in attn_decode_mfma_kernel<KV8> (same bytes, same scales),
// and this step attends over the quantised values.
typedef __attribute__((ext_vector_type(2))) float rt_f32x2;
template <int NW>
__global__ __launch_bounds__(64 * NW) void attn_decode_g1_fp8_kernel(DecodeFusedArgs a) {
  constexpr int D = 128;
  // NW waves per (batch, head), tiles dealt round-robin, merged through LDS: NW times the waves of
  // one-wave-per-row, so the last round of a 2560-row batch (2 waves per SIMD resident) is a
  // fraction of a row, not a whole one
  __shared__ float mrg[NW][2 + D];
  const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
  const int w = (int)(threadIdx.x >> 6);
  const int bh = blockIdx.x;
  const int b = bh / a.Hkv, hk = bh % a.Hkv;
  const int len = a.attn_len[b];
  const int s_new = a.slot[b];
  RT_ASSERT(len <= a.Smax && s_new >= 0 && s_new < a.Smax);
  int kbeg = a.kv_start ? a.kv_start[b] : 0;
  if (a.window > 0) kbeg = max(kbeg, len - a.window);
  const int p = a.pos ? a.pos[b] : 0;
  const bf16_t* row = a.qkv + (long)b * a.ldq;
  const unsigned char* kbase = (const unsigned char*)a.kc + (long)bh * a.Smax * D;
  const unsigned char* vbase = (const unsigned char*)a.vc + (long)bh * a.Smax * D;
  const float* ksb = a.ksc + (long)bh * a.SmaxP;
  const float* vsb = a.vsc + (long)bh * a.SmaxP;

  struct Tile { uint4 k0, k1; uint2 v[4]; float ks, vs; };
  auto load = [&](Tile& T, int c0) {
    const long key = min(c0 + r, len - 1);
    T.k0 = load_nt16(kbase + key * D + 32 * g);
    T.k1 = load_nt16(kbase + key * D + 32 * g + 16);
#pragma unroll
    for (int i = 0; i < 4; ++i) T.v[i] = load_nt8(vbase + (long)min(c0 + 4 * i + g, len - 1) * D + 8 * r);
    T.ks = ksb[key];
    T.vs = vsb[key];
  };
  Tile ta, tb, tc, td;
  constexpr int ST = 16 * NW;      // key stride between one wave's tiles
  const int cf = kbeg + 16 * w;  // this wave's tiles: cf + ST j
  if (cf < len) load(ta, cf);
  if (cf + ST < len) load(tb, cf + ST);
  if (cf + 2 * ST < len) load(tc, cf + 2 * ST);
  if (cf + 3 * ST < len) load(td, cf + 3 * ST);

  // ---- q / k_new / v_new (+ RoPE): lane group g holds chunks 4 s + g of q and k, chunk r of v
  const bool rot = a.cosT != nullptr;
  const bf16_t* qrow = row + (long)hk * D;
  const bf16_t* krow = row + (long)(a.Hq + hk) * D;
  const bf16_t* vrow = row + (long)(a.Hq + a.Hkv + hk) * D;
  uint4 qraw[4], kraw[4];
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) {
    qraw[s2] = *(const uint4*)(qrow + (4 * s2 + g) * 8);
    kraw[s2] = *(const uint4*)(krow + (4 * s2 + g) * 8);
  }
  const uint4 vx = *(const uint4*)(vrow + r * 8);
  float4 cq[2][2], sq[2][2];
  {
    const float* ct = rot ? a.cosT + (long)p * (D / 2) : (const float*)row;
    const float* stb = rot ? a.sinT + (long)p * (D / 2) : (const float*)row;
#pragma unroll
    for (int par = 0; par < 2; ++par) {
      const int j0 = (4 * par + g) * 8;
      cq[par][0] = *(const float4*)(ct + j0); cq[par][1] = *(const float4*)(ct + j0 + 4);
      sq[par][0] = *(const float4*)(stb + j0); sq[par][1] = *(const float4*)(stb + j0 + 4);
    }
  }
  auto rope8 = [&](const uint4& xv, const uint4& yv, const float4 (&c)[2], const float4 (&sn)[2], bool lo) -> uint4 {
    if (!rot) return xv;
    float x[8], y[8], o8[8];
    unpack8(xv, x);
    unpack8(yv, y);
    const float cs[8] = {c[0].x, c[0].y, c[0].z, c[0].w, c[1].x, c[1].y, c[1].z, c[1].w};
    const float sv[8] = {sn[0].x, sn[0].y, sn[0].z, sn[0].w, sn[1].x, sn[1].y, sn[1].z, sn[1].w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float t = a.sign * sv[e];
      o8[e] = fmaf(x[e], cs[e], lo ? -(y[e] * t) : y[e] * t);  // = rope_qkv_kernel's rounding
    }
    return pack8(o8);
  };
  float q[32];  // element 32 s + 8 g + e at q[8 s + e], times scale * log2 e
  uint4 knew[4];
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) {
    float f[8];
    unpack8(rope8(qraw[s2], qraw[s2 ^ 2], cq[s2 & 1], sq[s2 & 1], s2 < 2), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) q[8 * s2 + e] = f[e] * a.scale_log2;
    knew[s2] = rope8(kraw[s2], kraw[s2 ^ 2], cq[s2 & 1], sq[s2 & 1], s2 < 2);
  }
  // quantise k_new / v_new (absmax / 448 per head row), as attn_decode_mfma_kernel<KV8>
  uint2 kq[4], vq;
  float sk_new, sv_new;
  {
    float amk = 0.f, amv = 0.f, f[8];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      unpack8(knew[s2], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) amk = fmaxf(amk, fabsf(f[e]));
    }
    amk = fmaxf(amk, __shfl_xor(amk, 16, 64));
    amk = fmaxf(amk, __shfl_xor(amk, 32, 64));
    unpack8(vx, f);
#pragma unroll
    for (int e = 0; e < 8; ++e) amv = fmaxf(amv, fabsf(f[e]));
#pragma unroll
    for (int o2 = 1; o2 < 16; o2 <<= 1) amv = fmaxf(amv, __shfl_xor(amv, o2, 64));
    sk_new = amk > 0.f ? amk / 448.f : 1.f;
    sv_new = amv > 0.f ? amv / 448.f : 1.f;
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      unpack8(knew[s2], f);
      kq[s2] = f32x8_to_fp8(f, 1.f / sk_new);
    }
    unpack8(vx, f);
    vq = f32x8_to_fp8(f, 1.f / sv_new);
  }
  const bool has_new = s_new >= kbeg && s_new < len;
  if (has_new && w == 0) {
    unsigned char* kdst = (unsigned char*)a.kc + ((long)bh * a.Smax + s_new) * D;
    unsigned char* vdst = (unsigned char*)a.vc + ((long)bh * a.Smax + s_new) * D;
    if (r == 0) {
      *(uint4*)(kdst + 32 * g) = make_uint4(kq[0].x, kq[0].y, kq[1].x, kq[1].y);
      *(uint4*)(kdst + 32 * g + 16) = make_uint4(kq[2].x, kq[2].y, kq[3].x, kq[3].y);
    }
    if (g == 1) *(uint2*)(vdst + r * 8) = vq;
    if (lane == 0) {
      a.ksc[(long)bh * a.SmaxP + s_new] = sk_new;
      a.vsc[(long)bh * a.SmaxP + s_new] = sv_new;
    }
  }

  float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  auto consume = [&](const Tile& T, int c0) {
    unsigned kw[8] = {T.k0.x, T.k0.y, T.k0.z, T.k0.w, T.k1.x, T.k1.y, T.k1.z, T.k1.w};
    uint2 vv[4] = {T.v[0], T.v[1], T.v[2], T.v[3]};
    float ks = T.ks, vs = T.vs;
    if (has_new && s_new >= c0 && s_new < c0 + 16) {  // this step's own bytes and scales
      if (min(c0 + r, len - 1) == s_new) {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) { kw[2 * s2] = kq[s2].x; kw[2 * s2 + 1] = kq[s2].y; }
        ks = sk_new;
        vs = sv_new;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (min(c0 + 4 * i + g, len - 1) == s_new) vv[i] = vq;
    }
    float dot = 0.f;
#pragma unroll
    for (int w2 = 0; w2 < 8; ++w2) {
      const rt_f32x2 lo = __builtin_amdgcn_cvt_pk_f32_fp8(kw[w2], false);
      const rt_f32x2 hi = __builtin_amdgcn_cvt_pk_f32_fp8(kw[w2], true);
      dot = fmaf(q[4 * w2], lo.x, dot);
      dot = fmaf(q[4 * w2 + 1], lo.y, dot);
      dot = fmaf(q[4 * w2 + 2], hi.x, dot);
      dot = fmaf(q[4 * w2 + 3], hi.y, dot);
    }
    dot += __shfl_xor(dot, 16, 64);
    dot += __shfl_xor(dot, 32, 64);
    const float sc = c0 + r < len ? dot * ks : -INFINITY;
    float mx = sc;
#pragma unroll
    for (int o2 = 1; o2 < 16; o2 <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o2, 64));
    const float mn = fmaxf(m, mx);  // finite: every tile holds >= 1 valid key
    const float alpha = exp2f(m - mn);
    m = mn;
    const float pk = exp2f(sc - mn);
    float rs = pk;
#pragma unroll
    for (int o2 = 1; o2 < 16; o2 <<= 1) rs += __shfl_xor(rs, o2, 64);
    l = l * alpha + rs;
    const float pv = pk * vs;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] *= alpha;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float pp = __shfl(pv, 4 * i + g, 64);  // P' of key c0 + 4 i + g (lane r = 4 i + g)
      const rt_f32x2 v0 = __builtin_amdgcn_cvt_pk_f32_fp8(vv[i].x, false), v1 = __builtin_amdgcn_cvt_pk_f32_fp8(vv[i].x, true);
      const rt_f32x2 v2 = __builtin_amdgcn_cvt_pk_f32_fp8(vv[i].y, false), v3 = __builtin_amdgcn_cvt_pk_f32_fp8(vv[i].y, true);
      o[0] = fmaf(pp, v0.x, o[0]); o[1] = fmaf(pp, v0.y, o[1]);
      o[2] = fmaf(pp, v1.x, o[2]); o[3] = fmaf(pp, v1.y, o[3]);
      o[4] = fmaf(pp, v2.x, o[4]); o[5] = fmaf(pp, v2.y, o[5]);
      o[6] = fmaf(pp, v3.x, o[6]); o[7] = fmaf(pp, v3.y, o[7]);
    }
  };
  for (int c0 = cf; c0 < len; c0 += 4 * ST) {
    consume(ta, c0);
    if (c0 + 4 * ST < len) load(ta, c0 + 4 * ST);
    if (c0 + ST < len) {
      consume(tb, c0 + ST);
      if (c0 + 5 * ST < len) load(tb, c0 + 5 * ST);
    }
    if (c0 + 2 * ST < len) {
      consume(tc, c0 + 2 * ST);
      if (c0 + 6 * ST < len) load(tc, c0 + 6 * ST);
    }
    if (c0 + 3 * ST < len) {
      consume(td, c0 + 3 * ST);
      if (c0 + 7 * ST < len) load(td, c0 + 7 * ST);
    }
  }
  // the 4 lane groups hold disjoint key subsets of the same 8 dims
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    o[e] += __shfl_xor(o[e], 16, 64);
    o[e] += __shfl_xor(o[e], 32, 64);
  }
  // merge the waves' (m, l, O) (m = -inf, l = 0 for a wave without tiles)
  if (lane == 0) { mrg[w][0] = m; mrg[w][1] = l; }
  if (g == 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) mrg[w][2 + 8 * r + e] = o[e];
  }
  __syncthreads();
  if (w == 0 && g == 0) {
    float M = -INFINITY;
#pragma unroll
    for (int q2 = 0; q2 < NW; ++q2) M = fmaxf(M, mrg[q2][0]);
    float L = 0.f, y[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (M != -INFINITY) {
#pragma unroll
      for (int q2 = 0; q2 < NW; ++q2) {
        const float f = exp2f(mrg[q2][0] - M);  // 0 for a wave without tiles
        L += mrg[q2][1] * f;
#pragma unroll
        for (int e = 0; e < 8; ++e) y[e] += mrg[q2][2 + 8 * r + e] * f;
      }
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) y[e] *= inv;
    *(uint4*)(a.o + (long)b * a.ldo + (long)hk * D + 8 * r) = pack8(y);
  }
}

// ---------------------------------------------------------------------------------------------
// Fused decode step on MFMA (large batch: B * Hkv >= 256, one partition per (batch, kv head))
// ---------------------------------------------------------------------------------------------
// At batch 256 the decode attention of a layer streams ~250 MB of K/V (256 x 8 kv-heads x ~240
// keys x 512 B); the VALU kernel above spends ~120 instructions per key-lane on dot products,
// 16-lane shuffle reductions and the PV update (~3 TB/s). Here the G query heads of a kv head are
// the 16 "query rows" of the prefill kernel's swapped product (heads on the lane, G <= 16 valid).
// One wave per (batch, kv head); per 16-key tile:
//   * S^T = K·Q^T: 4 MFMAs whose K fragments are loaded straight from the cache into registers
//     (16 B per lane, no LDS); online softmax on 4 scores per lane (two cross-group shuffles);
//   * O += P·V: 8 MFMAs (K = 32: k-slots 4..7 are P = 0 against zero LDS rows), P = the packed
//     S^T accumulator, V through an LDS image (whole 256-B rows stored by ds_write_b128, read by
//     ds_read_b64_tr_b16).
// K and V of the next tile are prefetched into a second register set (plain loads only: no
// LDS-DMA, so hipcc's counted waits keep the prefetch in flight; 178 VGPRs = 2 waves per SIMD:
// all 2048 waves of a batch-256 layer are resident at once). The prologue issues every q / k_new /
// v_new / rotary-table load at once (one round trip) behind the first tile's loads. RoPE of q /
// k_new and the cache append are fused; lanes whose (clamped) key is the new token's slot use
// k_new / v_new from registers. Measured at batch 256 (Mistral-7B, 174..301 keys): 51 us per
// layer vs 80 us for the VALU kernel (profiles/decode_attn_r2_mfma.log).
//
// W > 1 (small batch, B * Hkv < 256 — the batch-1 RAG answer path): W waves share one (batch, kv
// head); wave w takes the 16-key tiles w, w + W, w + 2W, ... (its first two tiles' loads issued
// with the prologue's), and the W partial (m, l, O) states merge through LDS in the same launch —
// no cross-workgroup partition combine, so a layer's attention is one memory round trip plus a
// workgroup barrier instead of the split kernel's publish / ticket / merge chain.
// Long caches (a.NP > 1, a.PS keys per partition): B * Hkv * NP workgroups, partition `part`
// covering keys [part * PS, (part + 1) * PS) of the row; each publishes its merged (m, l, O) with
// write-through stores and takes a ticket, and the last of the row's NP partitions merges them —
// at 4k keys one workgroup per (batch, kv head) would stream 2 MB from one CU.
template <int G, int W, bool KV8 = false>
__global__ __launch_bounds__(64 * W) void attn_decode_mfma_kernel(DecodeFusedArgs a) {
  constexpr int D = 128, DS = D / 32, DT = D / 16;
  __shared__ __attribute__((aligned(16))) char vimg_all[W][32 * D * 2];  // per wave; rows 16..31 stay zero
  __shared__ __attribute__((aligned(16))) bf16_t qkv_st[(G + 2) * D];  // slab path (W == 1): reduced q | k | v
  const int lane = threadIdx.x & 63, g = lane >> 4, r16 = lane & 15;
  const int w = W > 1 ? (int)(threadIdx.x >> 6) : 0;
  char* vimg = vimg_all[w];
  // debug phase stamps (a.stamps: the launch's stamps argument): every load drained first
  auto stamp = [&](int k) {
    if (W > 1 && a.stamps) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      const long long t = __builtin_amdgcn_s_memrealtime();
      if (lane == 0) a.stamps[((long)blockIdx.x * W + w) * 8 + k] = t;
    }
  };
  stamp(0);
  const int NP = W > 1 ? max(a.NP, 1) : 1;
  const int part = blockIdx.x % NP, bh = blockIdx.x / NP;
  const int b = bh / a.Hkv, hk = bh % a.Hkv;
  const int len_row = a.attn_len[b];
  const int s_new = a.slot[b];
  RT_ASSERT(len_row <= a.Smax && s_new >= 0 && s_new < a.Smax);
  int kbeg = a.kv_start ? a.kv_start[b] : 0;
  if (a.window > 0) kbeg = max(kbeg, len_row - a.window);
  // this workgroup's keys [kbeg, len): the whole row, or partition `part` of it
  const int len = NP > 1 ? min(len_row, (part + 1) * a.PS) : len_row;
  if (NP > 1) kbeg = max(kbeg, part * a.PS);
  const int p = a.pos ? a.pos[b] : 0;
  const bf16_t* row = a.qkv + (long)b * a.ldq;
  const bf16_t* kbase = a.kc + ((long)b * a.Hkv + hk) * a.Smax * D;
  const bf16_t* vbase = a.vc + ((long)b * a.Hkv + hk) * a.Smax * D;
  // fp8 cache: byte rows of D, scales per slot
  const unsigned char* kbase8 = (const unsigned char*)a.kc + ((long)b * a.Hkv + hk) * a.Smax * D;
  const unsigned char* vbase8 = (const unsigned char*)a.vc + ((long)b * a.Hkv + hk) * a.Smax * D;
  const float* ksb = KV8 ? a.ksc + ((long)b * a.Hkv + hk) * a.SmaxP : nullptr;
  const float* vsb = KV8 ? a.vsc + ((long)b * a.Hkv + hk) * a.SmaxP : nullptr;

  // tile of 16 keys from c0 (32 registers per set: two sets keep every wave of a batch-256 layer
  // resident, 3 per SIMD): K fragments k[s] = K[c0 + r16][32 s + 8 g ..] (A operand of S^T);
  // V pieces v[i] = V[c0 + 4 i + g][8 r16 ..] (4 whole rows per load instruction).
  // Keys past len - 1 re-read slot len - 1 (masked).
  // fp8 tile (KV8): the lane's 32 K bytes (k-permuted row), 4 x 8 V bytes, and the scales of the
  // 4 keys c0 + 4 g + i whose scores the lane holds (S^T rows) — 24 registers instead of 32
  struct Tile16 { uint4 k[DS]; uint4 v[4]; };
  struct Tile8 { uint4 k8[2]; uint2 v8[4]; float ks[4], vs[4]; };
  typedef typename std::conditional<KV8, Tile8, Tile16>::type Tile;
  auto load = [&](Tile& T, int c0) {
    const long keyk = min(c0 + r16, len - 1);
    if constexpr (KV8) {
      T.k8[0] = load_nt16(kbase8 + keyk * D + 32 * g);
      T.k8[1] = load_nt16(kbase8 + keyk * D + 32 * g + 16);
#pragma unroll
      for (int i = 0; i < 4; ++i) T.v8[i] = load_nt8(vbase8 + (long)min(c0 + 4 * i + g, len - 1) * D + 8 * r16);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = min(c0 + 4 * g + i, len - 1);
        T.ks[i] = ksb[key];
        T.vs[i] = vsb[key];
      }
    } else if (a.kv_nt) {
#pragma unroll
      for (int s2 = 0; s2 < DS; ++s2) T.k[s2] = load_nt16(kbase + keyk * D + 32 * s2 + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) T.v[i] = load_nt16(vbase + (long)min(c0 + 4 * i + g, len - 1) * D + 8 * r16);
    } else {
#pragma unroll
      for (int s2 = 0; s2 < DS; ++s2) T.k[s2] = *(const uint4*)(kbase + keyk * D + 32 * s2 + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long key = min(c0 + 4 * i + g, len - 1);
        T.v[i] = *(const uint4*)(vbase + key * D + 8 * r16);
      }
    }
  };
  Tile ta, tb, tc;
  const int cfirst = kbeg + 16 * w, cstep = 16 * W;  // this wave's tiles: cfirst + j * cstep
  // fp8 tiles carry half the bytes: the single-wave kernel keeps THREE in flight (12 KiB per wave;
  // a fourth register set would cost the second wave per SIMD)
  constexpr bool DEEP8 = KV8 && W == 1;
  if (cfirst < len) load(ta, cfirst);
  if ((W > 1 || DEEP8) && cfirst + cstep < len) load(tb, cfirst + cstep);
  if ((W > 1 || DEEP8) && cfirst + 2 * cstep < len) load(tc, cfirst + 2 * cstep);

  // ---- q / k_new / v_new and the rotary tables, all loads at once. D = 128: chunk 4 s + g's
  // rotary partner (chunk ^ 8) is the lane's own chunk 4 (s ^ 2) + g, its table offset
  // ((chunk & 7) * 8) depends on s & 1 only ----
  const bool rot = a.cosT != nullptr;
  const bool has_new = s_new >= kbeg && s_new < len;
  const bf16_t* qrow = row + (long)min(hk * G + r16, a.Hq - 1) * D;
  const bf16_t* krow = row + (long)(a.Hq + hk) * D;
  const bf16_t* vrow = row + (long)(a.Hq + a.Hkv + hk) * D;
  if (a.qkv_slabs) {
    // split-K slabs of the qkv GEMM: this wave sums its (G + 2) x D slice once (in the order and
    // with the bf16 rounding of splitk_reduce_kernel) into LDS, and reads q / k / v from there
    constexpr int NCHK = (G + 2) * (D / 8);
    for (int ch = lane; ch < NCHK; ch += 64) {
      const int seg = ch / (D / 8), c8 = ch % (D / 8);
      const int head = seg < G ? hk * G + seg : (seg == G ? a.Hq + hk : a.Hq + a.Hkv + hk);
      float t8[8];
      sum_slabs8(a.qkv_slabs + (long)b * a.ldq + (long)head * D + c8 * 8, a.qkv_sstride, a.qkv_nsplit, t8);
      *(uint4*)(qkv_st + seg * D + c8 * 8) = pack8(t8);
    }
    qrow = qkv_st + min(r16, G - 1) * D;
    krow = qkv_st + G * D;
    vrow = qkv_st + (G + 1) * D;
  }
  uint4 qraw[DS], kraw[DS];
#pragma unroll
  for (int s2 = 0; s2 < DS; ++s2) {
    qraw[s2] = *(const uint4*)(qrow + (4 * s2 + g) * 8);
    kraw[s2] = *(const uint4*)(krow + (4 * s2 + g) * 8);
  }
  const uint4 vx = *(const uint4*)(vrow + r16 * 8);
  float4 cq[2][2], sq[2][2];
  {
    // unconditional (no branch between load batches): without tables read the qkv row
    const float* ct = rot ? a.cosT + (long)p * (D / 2) : (const float*)row;
    const float* stb = rot ? a.sinT + (long)p * (D / 2) : (const float*)row;
#pragma unroll
    for (int par = 0; par < 2; ++par) {
      const int j0 = (4 * par + g) * 8;
      cq[par][0] = *(const float4*)(ct + j0); cq[par][1] = *(const float4*)(ct + j0 + 4);
      sq[par][0] = *(const float4*)(stb + j0); sq[par][1] = *(const float4*)(stb + j0 + 4);
    }
  }
  // x rotated with partner y: lo half (chunk < 8) x c - y s', hi half x c + y s' (s' = sign sin),
  // rounded to bf16 as the unfused rope kernel stores it
  auto rope8 = [&](const uint4& xv, const uint4& yv, const float4 (&c)[2], const float4 (&sn)[2], bool lo) -> uint4 {
    if (!rot) return xv;
    float x[8], y[8], o8[8];
    unpack8(xv, x);
    unpack8(yv, y);
    const float cs[8] = {c[0].x, c[0].y, c[0].z, c[0].w, c[1].x, c[1].y, c[1].z, c[1].w};
    const float sv[8] = {sn[0].x, sn[0].y, sn[0].z, sn[0].w, sn[1].x, sn[1].y, sn[1].z, sn[1].w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float t = a.sign * sv[e];
      o8[e] = fmaf(x[e], cs[e], lo ? -(y[e] * t) : y[e] * t);  // = rope_qkv_kernel's rounding
    }
    return pack8(o8);
  };
  bf16x8 qf[DS];   // B operand of S^T = K·Q^T: Q[head r16][32 s + 8 g ..]
  uint4 knew[DS];  // rotated k_new chunks 4 s + g (the lane's K-fragment chunks)
#pragma unroll
  for (int s2 = 0; s2 < DS; ++s2) {
    const uint4 qv = rope8(qraw[s2], qraw[s2 ^ 2], cq[s2 & 1], sq[s2 & 1], s2 < 2);
    qf[s2] = __builtin_bit_cast(bf16x8, r16 < G ? qv : make_uint4(0, 0, 0, 0));
    knew[s2] = rope8(kraw[s2], kraw[s2 ^ 2], cq[s2 & 1], sq[s2 & 1], s2 < 2);
  }
  stamp(1);  // q / k_new / v_new / tables and the first tiles landed, RoPE done
  // fp8 cache: quantise k_new / v_new per (token, kv head) (absmax / 448); this step attends over
  // the quantised values too (knew / vxq hold them widened back to bf16, sk / sv their scales), so
  // the step sees exactly what later steps read from the cache
  uint4 vxq = vx;
  float sk_new = 1.f, sv_new = 1.f;
  uint2 kq[DS], vq = make_uint2(0, 0);
  if constexpr (KV8) {
    float amk = 0.f, amv = 0.f, f[8];
#pragma unroll
    for (int s2 = 0; s2 < DS; ++s2) {
      unpack8(knew[s2], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) amk = fmaxf(amk, fabsf(f[e]));
    }
    amk = fmaxf(amk, __shfl_xor(amk, 16, 64));  // lane group g holds chunks 4 s + g
    amk = fmaxf(amk, __shfl_xor(amk, 32, 64));
    unpack8(vx, f);
#pragma unroll
    for (int e = 0; e < 8; ++e) amv = fmaxf(amv, fabsf(f[e]));
#pragma unroll
    for (int o2 = 1; o2 < 16; o2 <<= 1) amv = fmaxf(amv, __shfl_xor(amv, o2, 64));  // chunk r16
    sk_new = amk > 0.f ? amk / 448.f : 1.f;
    sv_new = amv > 0.f ? amv / 448.f : 1.f;
    const float ik = 1.f / sk_new, iv = 1.f / sv_new;
#pragma unroll
    for (int s2 = 0; s2 < DS; ++s2) {
      unpack8(knew[s2], f);
      kq[s2] = f32x8_to_fp8(f, ik);
      knew[s2] = __builtin_bit_cast(uint4, fp8x8_to_bf16(kq[s2].x, kq[s2].y));
    }
    unpack8(vx, f);
    vq = f32x8_to_fp8(f, iv);
    vxq = __builtin_bit_cast(uint4, fp8x8_to_bf16(vq.x, vq.y));
  }
  // cache append: lane (g, 0) stores its 4 k chunks 4 s + g, lane group 1 the v chunks (wave 0)
  if (has_new && w == 0) {
    if constexpr (KV8) {
      unsigned char* kdst = (unsigned char*)a.kc + (((long)b * a.Hkv + hk) * a.Smax + s_new) * D;
      unsigned char* vdst = (unsigned char*)a.vc + (((long)b * a.Hkv + hk) * a.Smax + s_new) * D;
      if (r16 == 0) {  // k-permuted: chunks 4 s + g at bytes 32 g + 8 s
        *(uint4*)(kdst + 32 * g) = make_uint4(kq[0].x, kq[0].y, kq[1].x, kq[1].y);
        *(uint4*)(kdst + 32 * g + 16) = make_uint4(kq[2].x, kq[2].y, kq[3].x, kq[3].y);
      }
      if (g == 1) *(uint2*)(vdst + r16 * 8) = vq;
      if (lane == 0) {
        a.ksc[((long)b * a.Hkv + hk) * a.SmaxP + s_new] = sk_new;
        a.vsc[((long)b * a.Hkv + hk) * a.SmaxP + s_new] = sv_new;
      }
    } else {
      bf16_t* kdst = a.kc + (((long)b * a.Hkv + hk) * a.Smax + s_new) * D;
      bf16_t* vdst = a.vc + (((long)b * a.Hkv + hk) * a.Smax + s_new) * D;
      if (r16 == 0) {
#pragma unroll
        for (int s2 = 0; s2 < DS; ++s2) *(uint4*)(kdst + (4 * s2 + g) * 8) = knew[s2];
      }
      if (g == 1) *(uint4*)(vdst + r16 * 8) = vx;
    }
  }

  f32x4 o[DT];
#pragma unroll
  for (int c = 0; c < DT; ++c) o[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;  // of head r16 (identical over the 4 lane groups)
  // P·V runs K = 32 MFMAs on 16-key tiles: k-slots 4..7 carry P = 0 against zero V rows 16..31
#pragma unroll
  for (int i = 0; i < 4; ++i) *(uint4*)(vimg + v_off<D>(16 + 4 * i + g, r16)) = make_uint4(0, 0, 0, 0);

  auto consume = [&](Tile& T, int c0) {
    // bf16 K fragments / V pieces of the tile (fp8: widened, unscaled e4m3 values; the per-key
    // scales go on the scores and on P)
    uint4 kf[DS], vf[4];
    float ks[4] = {1.f, 1.f, 1.f, 1.f}, vs[4] = {1.f, 1.f, 1.f, 1.f};
    if constexpr (KV8) {
#pragma unroll
      for (int s2 = 0; s2 < DS; ++s2) {
        const uint4& q = T.k8[s2 >> 1];
        kf[s2] = __builtin_bit_cast(uint4, (s2 & 1) ? fp8x8_to_bf16(q.z, q.w) : fp8x8_to_bf16(q.x, q.y));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        vf[i] = __builtin_bit_cast(uint4, fp8x8_to_bf16(T.v8[i].x, T.v8[i].y));
        ks[i] = T.ks[i];
        vs[i] = T.vs[i];
      }
    } else {
#pragma unroll
      for (int s2 = 0; s2 < DS; ++s2) kf[s2] = T.k[s2];
#pragma unroll
      for (int i = 0; i < 4; ++i) vf[i] = T.v[i];
    }
    if (has_new && s_new >= c0 && s_new < c0 + 16) {
      if (min(c0 + r16, len - 1) == s_new) {
#pragma unroll
        for (int s2 = 0; s2 < DS; ++s2) kf[s2] = knew[s2];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (min(c0 + 4 * i + g, len - 1) == s_new) vf[i] = vxq;
        if (KV8 && c0 + 4 * g + i == s_new) {  // this step's own scales (the prefetched ones may be stale)
          ks[i] = sk_new;
          vs[i] = sv_new;
        }
      }
    }
    // V image rows 0..15 (the previous tile's transposed reads precede these writes in this
    // wave's LDS queue)
#pragma unroll
    for (int i = 0; i < 4; ++i) *(uint4*)(vimg + v_off<D>(4 * i + g, r16)) = vf[i];
    // S^T: lane holds the scores of keys c0 + 4 g + i for head r16
    f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < DS; ++s2)
      st = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kf[s2]), qf[s2], st, 0, 0, 0);
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = c0 + 4 * g + i < len ? st[i] * (KV8 ? ks[i] * a.scale_log2 : a.scale_log2) : -INFINITY;
      st[i] = x;
      mx = fmaxf(mx, x);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);  // finite: every tile holds >= 1 valid key
    const float alpha = exp2f(m - mn);
    m = mn;
    float rs = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float pv = exp2f(st[i] - mn);
      st[i] = KV8 ? pv * vs[i] : pv;  // fp8: the V scale of key c0 + 4 g + i rides on P
      rs += pv;
    }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    // O rows are heads 4 g + i: their factors live in lanes 4 g + i. Only rows < G are ever
    // stored or merged (an O row depends on its own P row only), so G < 4 rescales G rows
#pragma unroll
    for (int i = 0; i < (G < 4 ? G : 4); ++i) {
      const float al = __shfl(alpha, 4 * g + i, 64);
#pragma unroll
      for (int c = 0; c < DT; ++c) o[c][i] *= al;
    }
    // O += P·V: P (A operand) = the packed S^T accumulators, V (B operand) by transposed reads
    const bf16x8 pa = pack_bf16x8(st, f32x4{0.f, 0.f, 0.f, 0.f});
    const int qrow_ = lane >> 2 & 3, pcol = lane & 3;
#pragma unroll
    for (int c = 0; c < DT; ++c) {
      const int key_a = 4 * g + qrow_, col = 16 * c + 4 * pcol;
      const s16x4 lo = ds_tr16(vimg + v_off<D>(key_a, col >> 3) + ((col & 7) << 1));
      const s16x4 hi = ds_tr16(vimg + v_off<D>(key_a + 16, col >> 3) + ((col & 7) << 1));
      o[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, cat_tr(lo, hi), o[c], 0, 0, 0);
    }
  };

  if constexpr (W == 1 && !DEEP8) {
    for (int c0 = cfirst; c0 < len; c0 += 2 * cstep) {
      if (c0 + cstep < len) load(tb, c0 + cstep);
      consume(ta, c0);
      if (c0 + cstep < len) {
        if (c0 + 2 * cstep < len) load(ta, c0 + 2 * cstep);
        consume(tb, c0 + cstep);
      }
    }
  } else {
    // three tiles in flight (all of a wave's tiles at up to 24 W keys: one memory round trip);
    // a register set is refilled right after its tile is consumed
    for (int c0 = cfirst; c0 < len; c0 += 3 * cstep) {
      consume(ta, c0);
      if (c0 + 3 * cstep < len) load(ta, c0 + 3 * cstep);
      if (c0 + cstep < len) {
        consume(tb, c0 + cstep);
        if (c0 + 4 * cstep < len) load(tb, c0 + 4 * cstep);
      }
      if (c0 + 2 * cstep < len) {
        consume(tc, c0 + 2 * cstep);
        if (c0 + 5 * cstep < len) load(tc, c0 + 5 * cstep);
      }
    }
  }
  if constexpr (W == 1) {
    // ---- normalise and store: lane holds O[head 4 g + i][d = 16 c + r16] ----
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int h = 4 * g + i;
      const float lh = __shfl(l, h, 64);
      const float inv = lh > 0.f ? 1.f / lh : 0.f;
      if (h < G) {
        bf16_t* orow = a.o + (long)b * a.ldo + (long)(hk * G + h) * D;
#pragma unroll
        for (int c = 0; c < DT; ++c) orow[16 * c + r16] = f2bf(o[c][i] * inv);
      }
    }
  } else {
    stamp(2);  // this wave's tiles consumed
    // ---- merge the W waves' states (m = -inf, l = 0 for a wave without tiles) ----
    __shared__ float mst[W][16], lst[W][16];
    __shared__ float ost[W][G][D];
    if (g == 0) {
      mst[w][r16] = m;
      lst[w][r16] = l;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int h = 4 * g + i;
      if (h < G) {
#pragma unroll
        for (int c = 0; c < DT; ++c) ost[w][h][16 * c + r16] = o[c][i];
      }
    }
    __syncthreads();
    float* pp = NP > 1 ? a.part + (long)bh * NP * G * (D + 2) : nullptr;
    for (int e = threadIdx.x; e < G * D; e += 64 * W) {
      const int h = e / D, d = e % D;
      float M = -INFINITY;
#pragma unroll
      for (int q = 0; q < W; ++q) M = fmaxf(M, mst[q][h]);
      float L = 0.f, O = 0.f;
      if (M != -INFINITY) {
#pragma unroll
        for (int q = 0; q < W; ++q) {
          const float mq = mst[q][h];
          if (mq == -INFINITY) continue;
          const float f = exp2f(mq - M);
          L += lst[q][h] * f;
          O += ost[q][h][d] * f;
        }
      }
      if (NP > 1) {  // publish the unnormalised partial (write-through stores)
        float* r = pp + ((long)part * G + h) * (D + 2);
        __hip_atomic_store(r + d, O, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d == 0) {
          __hip_atomic_store(r + D, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(r + D + 1, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        a.o[(long)b * a.ldo + (long)(hk * G + h) * D + d] = f2bf(L > 0.f ? O / L : 0.f);
      }
    }
    if (NP > 1) {
      // drained payload -> ticket (handoff-flag); the row's last partition merges all NP records
      __shared__ int last_flag;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        const unsigned old = __hip_atomic_fetch_add(a.tickets + bh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_flag = old == (unsigned)(NP - 1);
      }
      __syncthreads();
      if (!last_flag) return;
      for (int e = threadIdx.x; e < G * D; e += 64 * W) {
        const int h = e / D, d = e % D;
        float M = -INFINITY, L = 0.f, O = 0.f;
#pragma unroll 4
        for (int q = 0; q < NP; ++q) {
          const float* r = pp + ((long)q * G + h) * (D + 2);
          const float mq = __hip_atomic_load(r + D, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (mq == -INFINITY) continue;  // empty partition: o[] never written
          const float lq = __hip_atomic_load(r + D + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const float oq = __hip_atomic_load(r + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const float Mn = fmaxf(M, mq);
          const float r0 = exp2f(M - Mn), r1 = exp2f(mq - Mn);
          L = L * r0 + lq * r1;
          O = O * r0 + oq * r1;
          M = Mn;
        }
        a.o[(long)b * a.ldo + (long)(hk * G + h) * D + d] = f2bf(L > 0.f ? O / L : 0.f);
      }
      if (threadIdx.x == 0) __hip_atomic_store(a.tickets + bh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    stamp(3);
  }
}

// ---------------------------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------------------------
struct AttnBwdArgs {
  const bf16_t* q; long ldq;
  const bf16_t* k; long ldk;
  const bf16_t* v; long ldv;
  const bf16_t* o; long ldo;
  const bf16_t* dout; long lddo;
  const float* lse;            // [B, Hq, S]
  float* delta;                // [B, Hq, S]
  float* dq;                   // fp32 [B*S, Hq*D] (zeroed; atomic form only)
  bf16_t* dqb; long lddq;      // bf16 dQ (separate dQ kernel)
  bf16_t* dk; long lddk;       // may alias into a d_qkv buffer
  bf16_t* dv; long lddv;
  const int* kv_start;
  int B, S, Hq, Hkv;
  int causal, window;
  float scale_log2;            // scale * log2 e
  float scale;
  int lpt;                     // heaviest-first dispatch order (attn_block_xyz; causal grids)
  // RoPE backward fused into the dQ / dK stores (null: none): q / k were rotated by angle row
  // rope_pos[b * S + s] of the [positions, D / 2] tables; dq / dk are inverse-rotated from their
  // bf16-rounded values with rope_qkv_kernel's arithmetic (sign -1): bitwise the separate pass
  const int* rope_pos;
  const float* rope_cos;
  const float* rope_sin;
};

// inverse rotation of one (first-half, second-half) pair of a bf16-rounded gradient: x1 / x2 are
// the rounded values at dims e / e + D/2; rope_qkv_kernel with sign = -1
__device__ __forceinline__ void rope_bwd_pair(float x1, float x2, float c, float sn, float& o1, float& o2) {
  const float s = -sn;
  o1 = fmaf(x1, c, -(x2 * s));
  o2 = fmaf(x2, c, x1 * s);
}

template <int D>
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(AttnBwdArgs a) {
  // delta[b,h,q] = sum_d dO*O: LPR = D/8 lanes per (token, head) row, one 16-B load per operand
  // per lane (a wave covers 64 / LPR rows; the former one-row-per-wave, 4-B-per-lane version ran
  // at a third of the copy bandwidth)
  constexpr int LPR = D / 8, RPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const long row = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  const long total = (long)a.B * a.S * a.Hq;
  const int c = lane % LPR;
  float s = 0.f;
  if (row < total) {
    const int h = row % a.Hq;
    const long t = row / a.Hq;  // b*S + q
    float o8[8], g8[8];
    unpack8(*(const uint4*)(a.o + t * a.ldo + (long)h * D + c * 8), o8);
    unpack8(*(const uint4*)(a.dout + t * a.lddo + (long)h * D + c * 8), g8);
#pragma unroll
    for (int e = 0; e < 8; ++e) s += o8[e] * g8[e];
  }
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (row < total && c == 0) {
    const int h = row % a.Hq;
    const long t = row / a.Hq;
    const long b = t / a.S, q = t % a.S;
    a.delta[(b * a.Hq + h) * a.S + q] = s;
  }
}

template <int D>
__global__ __launch_bounds__(256, 2) void attn_bwd_kernel(AttnBwdArgs a) {
  constexpr int NCH = D / 8, DS = D / 32, DT = D / 16;
  constexpr int TB = 64 * D * 2;
  // LDS: Q tile | dO tile | lse[64] | delta[64] (dQ is the separate attn_bwd_dq_kernel: no K or dS
  // tile here)
  __shared__ __attribute__((aligned(16))) char smem[2 * TB + 2 * 64 * 4];
  char* Qs = smem;
  char* Os = smem + TB;  // dO
  float* lse_s = (float*)(smem + 2 * TB);
  float* del_s = lse_s + 64;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int3 bx = attn_block_xyz(a.lpt ? 2 : 0);  // key blocks: the lowest sees the most queries
  const int b = bx.z, hk = bx.y;
  const int kb0 = bx.x * 64;
  const int G = a.Hq / a.Hkv;
  const int start = a.kv_start ? a.kv_start[b] : 0;
  const int mykey = kb0 + wid * 16 + r16;  // this lane's key column
  constexpr int CPT = 64 * NCH / 256;

  // this wave's K, V fragments (B operands) -> registers
  bf16x8 kf[DS], vf[DS];
  {
    const int kk = min(mykey, a.S - 1);
#pragma unroll
    for (int s = 0; s < DS; ++s) {
      kf[s] = *(const bf16x8*)(a.k + ((long)b * a.S + kk) * a.ldk + (long)hk * D + 32 * s + 8 * g);
      vf[s] = *(const bf16x8*)(a.v + ((long)b * a.S + kk) * a.ldv + (long)hk * D + 32 * s + 8 * g);
    }
  }
  // retire these loads once, here (else hipcc re-waits vmcnt(0) for them inside the loop, which
  // also drains the Q/dO prefetch and the dQ atomics every iteration)
#pragma unroll
  for (int s = 0; s < DS; ++s) asm volatile("" : "+v"(kf[s]), "+v"(vf[s]));
  f32x4 dk[DT], dvv[DT];
#pragma unroll
  for (int c = 0; c < DT; ++c) { dk[c] = f32x4{0.f, 0.f, 0.f, 0.f}; dvv[c] = f32x4{0.f, 0.f, 0.f, 0.f}; }

  int qbeg = a.causal ? kb0 : 0;
  qbeg = max(qbeg, start) & ~63;
  int qend = a.S;
  if (a.window > 0) qend = min(qend, kb0 + 63 + a.window);
  const bool key_valid = mykey >= start && mykey < a.S;

  // (head, q-tile) iterations, flattened; the next one's Q / dO tile, lse and delta are prefetched
  // into registers while the current one computes (staged to LDS after the loop-top barrier)
  const int nqt = qend > qbeg ? (qend - qbeg + 63) / 64 : 0;
  const int nit = G * nqt;
  const int lc = tid % NCH, lrow = tid / NCH;
  constexpr int RSTEP = 256 / NCH;
  u32x4 qreg[CPT], oreg[CPT];
  float lse_r = 0.f, del_r = 0.f;  // raw loads: scaled / masked only when staged (no early wait)
  bool row_ok = false;
  auto load_qdo = [&](int it) {
    const int h = hk * G + it / nqt, qt = qbeg + (it % nqt) * 64;
    const bf16_t* qb = a.q + (long)b * a.S * a.ldq + (long)h * D + lc * 8;
    const bf16_t* ob = a.dout + (long)b * a.S * a.lddo + (long)h * D + lc * 8;
#pragma unroll
    for (int r = 0; r < CPT; ++r) {
      const long qq = min(qt + lrow + RSTEP * r, a.S - 1);
      qreg[r] = *(const u32x4*)(qb + qq * a.ldq);
      oreg[r] = *(const u32x4*)(ob + qq * a.lddo);
    }
    if (tid < 64) {
      const int qq = qt + tid;
      row_ok = qq < a.S;
      const long li = ((long)b * a.Hq + h) * a.S + min(qq, a.S - 1);
      lse_r = a.lse[li];
      del_r = a.delta[li];
    }
  };
  if (nit > 0) load_qdo(0);

  for (int it = 0; it < nit; ++it) {
    const int h = hk * G + it / nqt, qt = qbeg + (it % nqt) * 64;
    {
      __syncthreads();  // previous users of Q/dO/dS tiles are done
#pragma unroll
      for (int r = 0; r < CPT; ++r) {
        *(u32x4*)(Qs + k_off<D>(lrow + RSTEP * r, lc)) = qreg[r];
        *(u32x4*)(Os + k_off<D>(lrow + RSTEP * r, lc)) = oreg[r];
      }
      if (tid < 64) {
        lse_s[tid] = row_ok ? lse_r * 1.4426950408889634f : INFINITY;
        del_s[tid] = row_ok ? del_r : 0.f;
      }
      __syncthreads();
      if (it + 1 < nit) load_qdo(it + 1);

      // S[q][key] and dP[q][key] for 4 q-subtiles (key on lane)
      f32x4 sp[4], dp[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        sp[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < DS; ++s) {
          const bf16x8 qa = *(const bf16x8*)(Qs + k_off<D>(16 * u + r16, 4 * s + g));
          const bf16x8 oa = *(const bf16x8*)(Os + k_off<D>(16 * u + r16, 4 * s + g));
          sp[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kf[s], sp[u], 0, 0, 0);
          dp[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa, vf[s], dp[u], 0, 0, 0);
        }
      }
      // P and dS (element (u,i) <-> q = qt + 16u + 4g + i, key = mykey)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ql = 16 * u + 4 * g + i;
          const int qq = qt + ql;
          bool ok = key_valid && qq < a.S;
          if (a.causal) ok = ok && mykey <= qq;
          if (a.window > 0) ok = ok && (qq - mykey) < a.window;
          const float p = ok ? exp2f(sp[u][i] * a.scale_log2 - lse_s[ql]) : 0.f;
          sp[u][i] = p;
          dp[u][i] = p * (dp[u][i] - del_s[ql]);
        }
      // dV^T += dO^T · P ; dK^T += Q^T · dS  (A via transposed reads, B = accumulators)
      const int qrow = lane >> 2 & 3, pcol = lane & 3;
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        const bf16x8 pb = pack_bf16x8(sp[2 * qs], sp[2 * qs + 1]);
        const bf16x8 db = pack_bf16x8(dp[2 * qs], dp[2 * qs + 1]);
#pragma unroll
        for (int c = 0; c < DT; ++c) {
          const int rowa = 32 * qs + 4 * g + qrow;
          const int col = 16 * c + 4 * pcol;
          // Q and dO tiles use the K-style image: tr reads address it with the same k_off
          const bf16x8 oT = cat_tr(ds_tr16(Os + k_off<D>(rowa, col >> 3) + ((col & 7) << 1)),
                                   ds_tr16(Os + k_off<D>(rowa + 16, col >> 3) + ((col & 7) << 1)));
          const bf16x8 qT = cat_tr(ds_tr16(Qs + k_off<D>(rowa, col >> 3) + ((col & 7) << 1)),
                                   ds_tr16(Qs + k_off<D>(rowa + 16, col >> 3) + ((col & 7) << 1)));
          dvv[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oT, pb, dvv[c], 0, 0, 0);
          dk[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qT, db, dk[c], 0, 0, 0);
        }
      }
    }
  }
  // write dK, dV (lane holds dX^T[d = 16c + 4g + i][key = mykey]; dims d and d + D/2 are
  // fragments c and c + DT/2 of the same lane: the RoPE backward pairs them in registers)
  if (mykey < a.S) {
    bf16_t* dkrow = a.dk + ((long)b * a.S + mykey) * a.lddk + (long)hk * D;
    if (a.rope_cos) {
      const long tb = (long)a.rope_pos[(long)b * a.S + mykey] * (D / 2);
#pragma unroll
      for (int c = 0; c < DT / 2; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int d = 16 * c + 4 * g + i;
          float o1, o2;
          rope_bwd_pair(bf2f(f2bf(dk[c][i] * a.scale)), bf2f(f2bf(dk[c + DT / 2][i] * a.scale)), a.rope_cos[tb + d],
                        a.rope_sin[tb + d], o1, o2);
          dkrow[d] = f2bf(o1);
          dkrow[d + D / 2] = f2bf(o2);
        }
    } else {
#pragma unroll
      for (int c = 0; c < DT; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i) dkrow[16 * c + 4 * g + i] = f2bf(dk[c][i] * a.scale);
    }
#pragma unroll
    for (int c = 0; c < DT; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a.dv[((long)b * a.S + mykey) * a.lddv + (long)hk * D + 16 * c + 4 * g + i] = f2bf(dvv[c][i]);
  }
}

// dQ without atomics: one workgroup = 64 query rows of one (batch, head), 4 waves x 16 rows (the
// forward's swapped geometry). Per 64-key tile (K and V register-prefetched into K-style LDS
// images): S^T = K·Q^T and dP^T = V·dO^T with the key on the MFMA row and the query on the lane;
// P = exp2(S·scale·log2e − lse·log2e) (no online softmax: lse is known), dS = P (dP − delta),
// masks; dQ += dS·K with dS (packed accumulators) as the A operand and K^T by transposed reads of
// the same K image. Each dQ element is written once, in bf16 (the atomic form added one fp32 row
// per key block: ~0.5 GB of atomics per Mistral-7B layer at 9.6k tokens, bound at ~1.3 TB/s).
// HP (GQA-4, causal, short sequences): a workgroup = 16 positions x the 4 query heads of one kv
// head (wave w = head 4 hk + w), every wave on the same causal key range and one K / V staging for
// the 4 heads; per row the same key tiles in the same order (trailing fully masked tiles add exact
// zeros), so dQ is bitwise the 64-row form's.
template <int D, bool HP = false>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(AttnBwdArgs a) {
  constexpr int NCH = D / 8, DS = D / 32, DT = D / 16;
  constexpr int TILE_BYTES = 64 * D * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE_BYTES];
  char* Ks = smem;
  char* Vs = smem + TILE_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int3 bx = attn_block_xyz(a.lpt);
  const int b = bx.z;
  const int h = HP ? bx.y * 4 + wid : bx.y;
  const int hk = HP ? bx.y : h / (a.Hq / a.Hkv);
  constexpr int QROWS = HP ? 16 : 64;
  const int qblk0 = bx.x * QROWS;
  const int q0 = HP ? qblk0 : qblk0 + wid * 16;
  const int start = a.kv_start ? a.kv_start[b] : 0;
  int kend = a.S;
  if (a.causal) kend = min(kend, min(qblk0 + QROWS - 1, a.S - 1) + 1);
  int kbeg = start;
  if (a.window > 0) kbeg = max(kbeg, qblk0 - a.window + 1);
  kbeg = max(kbeg, 0) & ~63;

  // Q and dO fragments (B operands): lane holds X[q0 + r16][32 s + 8 g .. +8]
  const int qrow = min(q0 + r16, a.S - 1);
  bf16x8 qf[DS], of[DS];
  {
    const bf16_t* qp = a.q + ((long)b * a.S + qrow) * a.ldq + (long)h * D + 8 * g;
    const bf16_t* op = a.dout + ((long)b * a.S + qrow) * a.lddo + (long)h * D + 8 * g;
#pragma unroll
    for (int s2 = 0; s2 < DS; ++s2) {
      qf[s2] = *(const bf16x8*)(qp + 32 * s2);
      of[s2] = *(const bf16x8*)(op + 32 * s2);
    }
  }
  const long li = ((long)b * a.Hq + h) * a.S + qrow;
  const float lse2 = a.lse[li] * 1.4426950408889634f, del = a.delta[li];
  // retire these loads here (else hipcc re-waits vmcnt(0) for them inside the loop)
#pragma unroll
  for (int s2 = 0; s2 < DS; ++s2) asm volatile("" : "+v"(qf[s2]), "+v"(of[s2]));

  f32x4 dq[DT];
#pragma unroll
  for (int c = 0; c < DT; ++c) dq[c] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int CPT = 64 * NCH / 256;  // 16-B chunks per thread per tile
  constexpr int KSTEP = 256 / NCH;
  const int lc = tid % NCH, lkey = tid / NCH;
  const bf16_t* kb = a.k + (long)b * a.S * a.ldk + (long)hk * D + lc * 8;
  const bf16_t* vb = a.v + (long)b * a.S * a.ldv + (long)hk * D + lc * 8;
  u32x4 kreg[CPT], vreg[CPT];
  auto load_tile = [&](int kv0) {
#pragma unroll
    for (int r = 0; r < CPT; ++r) {
      const long kk = min(kv0 + lkey + KSTEP * r, a.S - 1);
      kreg[r] = *(const u32x4*)(kb + kk * a.ldk);
      vreg[r] = *(const u32x4*)(vb + kk * a.ldv);
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int r = 0; r < CPT; ++r) {
      *(u32x4*)(Ks + k_off<D>(lkey + KSTEP * r, lc)) = kreg[r];
      *(u32x4*)(Vs + k_off<D>(lkey + KSTEP * r, lc)) = vreg[r];
    }
  };
  if (kbeg < kend) {
    load_tile(kbeg);
    store_tile();
  }
  __syncthreads();

  const int qq = q0 + r16;  // this lane's query row
  for (int kv0 = kbeg; kv0 < kend; kv0 += 64) {
    const bool has_next = kv0 + 64 < kend;
    if (has_next) load_tile(kv0 + 64);
    // S^T[t], dP^T[t]: lane holds (key kv0 + 16 t + 4 g + i, query qq)
    f32x4 st[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < DS; ++s2) {
        const bf16x8 kf = *(const bf16x8*)(Ks + k_off<D>(16 * t + r16, 4 * s2 + g));
        const bf16x8 vf = *(const bf16x8*)(Vs + k_off<D>(16 * t + r16, 4 * s2 + g));
        st[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[s2], st[t], 0, 0, 0);
        dp[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, of[s2], dp[t], 0, 0, 0);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int kk = kv0 + 16 * t + 4 * g + i;
        bool ok = kk >= start && kk < a.S && qq < a.S;
        if (a.causal) ok = ok && kk <= qq;
        if (a.window > 0) ok = ok && (qq - kk) < a.window;
        const float pv = ok ? exp2f(st[t][i] * a.scale_log2 - lse2) : 0.f;
        st[t][i] = pv * (dp[t][i] - del);  // dS^T
      }
    // dQ += dS · K: A = packed dS^T accumulators [q][keys], B = K^T by transposed reads
    const int qr = lane >> 2 & 3, pcol = lane & 3;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 da = pack_bf16x8(st[2 * ks], st[2 * ks + 1]);
#pragma unroll
      for (int c = 0; c < DT; ++c) {
        const int key_a = 32 * ks + 4 * g + qr, col = 16 * c + 4 * pcol;
        const s16x4 lo = ds_tr16(Ks + k_off<D>(key_a, col >> 3) + ((col & 7) << 1));
        const s16x4 hi = ds_tr16(Ks + k_off<D>(key_a + 16, col >> 3) + ((col & 7) << 1));
        dq[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, cat_tr(lo, hi), dq[c], 0, 0, 0);
      }
    }
    __syncthreads();
    if (has_next) store_tile();
    __syncthreads();
  }
  // lane holds dQ[q0 + 4 g + i][16 c + r16] (dims d and d + D/2: fragments c and c + DT/2)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qo = q0 + 4 * g + i;
    if (qo < a.S) {
      bf16_t* dst = a.dqb + ((long)b * a.S + qo) * a.lddq + (long)h * D;
      if (a.rope_cos) {
        const long tb = (long)a.rope_pos[(long)b * a.S + qo] * (D / 2);
#pragma unroll
        for (int c = 0; c < DT / 2; ++c) {
          const int d = 16 * c + r16;
          float o1, o2;
          rope_bwd_pair(bf2f(f2bf(dq[c][i] * a.scale)), bf2f(f2bf(dq[c + DT / 2][i] * a.scale)), a.rope_cos[tb + d],
                        a.rope_sin[tb + d], o1, o2);
          dst[d] = f2bf(o1);
          dst[d + D / 2] = f2bf(o2);
        }
      } else {
#pragma unroll
        for (int c = 0; c < DT; ++c) dst[16 * c + r16] = f2bf(dq[c][i] * a.scale);
      }
    }
  }
}

}  // namespace rt

using namespace rt;

// heaviest-first dispatch (attn_block_xyz) on causal grids of at most tuning().attn_lpt workgroups
// (32 per CU): at the PPO update's minibatch it trims the launch tail (profiles/r6/attn_lpt_ab.log:
// forward -3..5 %, backward -7..9 %); on 4x larger grids (reference scoring, prefill) it was slower
// (+1..7 %): consecutive workgroups of an XCD then span too many kv heads for its L2
static int attn_lpt_on(dim3 grid, int causal) {
  const long nwg = (long)grid.x * grid.y * grid.z;
  return causal && grid.x > 1 && nwg <= tuning().attn_lpt ? 1 : 0;
}

extern "C" int rt_attn_fwd(const void* q, long ldq, const void* k, long ldk, const void* v, long ldv, void* o, long ldo,
                           float* lse, const int* kv_start, const int* kv_len, const float* rel_bias, int rb_L, int B,
                           int Sq, int Sk, int Hq, int Hkv, int D, int causal, int window, float scale,
                           hipStream_t stream) {
  AttnArgs a;
  a.q = (const bf16_t*)q; a.ldq = ldq; a.k = (const bf16_t*)k; a.ldk = ldk; a.v = (const bf16_t*)v; a.ldv = ldv;
  a.o = (bf16_t*)o; a.ldo = ldo; a.lse = lse; a.kv_start = kv_start; a.kv_len = kv_len; a.rel_bias = rel_bias;
  a.rb_L = rb_L; a.B = B; a.Sq = Sq; a.Sk = Sk; a.Hq = Hq; a.Hkv = Hkv; a.causal = causal; a.window = window;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.lpt = 0;
  if (B == 0 || Sq == 0) return 0;
  // GQA (4 query heads per kv head), D = 128, short sequences: the head-packed 32-position tiles
  // (every wave of a workgroup on the same causal key range)
  if (D == 128 && Hkv * 4 == Hq && causal && Sq <= tuning().attn_fwd_hp_maxs && !rel_bias) {
    dim3 grid((Sq + 31) / 32, Hkv, B), block(256);
    a.lpt = attn_lpt_on(grid, causal);
    hipLaunchKernelGGL((attn_fwd_kernel<128, 2, true>), grid, block, 0, stream, a);
    RT_LAUNCH_CHECK();
    return 0;
  }
  // other head groupings (MHA), D = 128: 64-position tiles of one head (4 waves x 16 rows)
  if (D == 128 && causal && Sq <= tuning().attn_fwd_hp_maxs && !rel_bias) {
    dim3 grid((Sq + 63) / 64, Hq, B), block(256);
    a.lpt = attn_lpt_on(grid, causal);
    hipLaunchKernelGGL((attn_fwd_kernel<128, 1, false, true>), grid, block, 0, stream, a);
    RT_LAUNCH_CHECK();
    return 0;
  }
  dim3 grid((Sq + 127) / 128, Hq, B), block(256);
  a.lpt = attn_lpt_on(grid, causal);
  switch (D) {
    case 32: hipLaunchKernelGGL(attn_fwd_kernel<32>, grid, block, 0, stream, a); break;
    case 64: hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, block, 0, stream, a); break;
    case 128: hipLaunchKernelGGL(attn_fwd_kernel<128>, grid, block, 0, stream, a); break;
    default: return -1;
  }
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_attn_decode(const void* q, long ldq, const void* kc, const void* vc, int Smax, const int* kv_len,
                              const int* kv_start, int window, float* part, int NP, int PS, void* o, long ldo, int B,
                              int Hq, int Hkv, int D, float scale, hipStream_t stream) {
  DecodeArgs a;
  a.q = (const bf16_t*)q; a.ldq = ldq; a.kc = (const bf16_t*)kc; a.vc = (const bf16_t*)vc; a.Smax = Smax;
  a.kv_len = kv_len; a.kv_start = kv_start; a.window = window; a.part = part; a.o = (bf16_t*)o; a.ldo = ldo;
  a.B = B; a.Hq = Hq; a.Hkv = Hkv; a.NP = NP; a.PS = PS; a.scale_log2 = scale * 1.4426950408889634f;
  const int G = Hq / Hkv;
  if (B == 0) return 0;
  dim3 grid(NP, Hkv, B), block(256);
  const size_t shm = (size_t)(G * PS + 4 * G * D) * sizeof(float);
#define DEC_CASE(DD, GG)                                                                      \
  if (D == DD && G == GG) {                                                                   \
    hipLaunchKernelGGL((attn_decode_kernel<DD, GG>), grid, block, shm, stream, a);            \
    hipLaunchKernelGGL((attn_decode_combine_kernel<DD, GG>), dim3(Hkv, B), dim3(256), 0, stream, a); \
    RT_LAUNCH_CHECK();                                                                        \
    return 0;                                                                                 \
  }
  DEC_CASE(128, 1) DEC_CASE(128, 2) DEC_CASE(128, 4) DEC_CASE(128, 8)
  DEC_CASE(64, 1) DEC_CASE(64, 2) DEC_CASE(64, 4) DEC_CASE(64, 8)
  DEC_CASE(32, 1)
#undef DEC_CASE
  return -1;
}

// keys per chunk of the fused kernel: 4 waves x (64 / (D/8)) keys per step x NK (= 4)
extern "C" int rt_attn_decode_fused_ps(int D, int nk) { return 4 * (64 / (D / 8)) * nk; }

// waves per (batch, kv head) of the small-batch MFMA decode attention. Caches up to 1024 slots run
// one workgroup per (batch, kv head) (<= 8 tiles per wave: the 3-tile register prefetch covers the
// memory round trip); longer caches split the row into partitions of about RT_DECODE_MW_KPP (512)
// keys, at most the workspace's NP, merged by the last arriving partition.
constexpr int DEC_MW = 8;
static bool rt_attn_decode_mw_ok(int B, int Hq, int Hkv, int D, int Smax) {
  const int G = Hkv ? Hq / Hkv : 0;
  return D == 128 && (long)B * Hkv < std::max(256, tuning().decode_mw_bh) && (G == 1 || G == 2 || G == 4 || G == 8);
}
static int rt_attn_decode_mw_np(int Smax, int np_ws) {
  const int kpp = std::max(16, tuning().decode_mw_kpp);
  if (Smax <= tuning().decode_mw_smax || np_ws <= 1) return 1;
  return std::max(1, std::min(np_ws, (Smax + kpp - 1) / kpp));
}
extern "C" int rt_attn_decode_mfma_ok(int B, int Hq, int Hkv, int D, int NP) {
  const int G = Hkv ? Hq / Hkv : 0;
  return NP == 1 && D == 128 && (long)B * Hkv >= std::max(256, tuning().decode_mw_bh) &&
         (G == 1 || G == 2 || G == 4 || G == 8 || G == 16);
}

// Prompt K / V (rows [b * S + s] of the rotated qkv) -> fp8 cache slots [0, S): one 16-lane group
// per (token, kv head, K | V), 8 elements per lane, absmax over the head row by shuffles. K rows
// are written k-permuted (chunk c = 4 s + g at byte 32 g + 8 s), as attn_decode_mfma_kernel<KV8>
// reads them. D = 128.
__global__ __launch_bounds__(256) void kv_store_fp8_kernel(const bf16_t* __restrict__ qkv, long ldq,
                                                           unsigned char* __restrict__ kc, unsigned char* __restrict__ vc,
                                                           float* __restrict__ ksc, float* __restrict__ vsc, int B, int S,
                                                           int Hq, int Hkv, int Smax, int SmaxP) {
  constexpr int D = 128;
  const long gid = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int c = threadIdx.x & 15;
  if (gid >= (long)B * S * Hkv * 2) return;  // whole 16-lane groups
  const int kv = (int)(gid & 1);
  const long t = gid >> 1;
  const int hk = (int)(t % Hkv);
  const long row = t / Hkv;
  const int b = (int)(row / S), s = (int)(row % S);
  float f[8];
  unpack8(*(const uint4*)(qkv + row * ldq + (long)(Hq + kv * Hkv + hk) * D + 8 * c), f);
  float am = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(f[e]));
#pragma unroll
  for (int o2 = 1; o2 < 16; o2 <<= 1) am = fmaxf(am, __shfl_xor(am, o2, 16));
  const float sc = am > 0.f ? am / 448.f : 1.f;
  const uint2 q = f32x8_to_fp8(f, 1.f / sc);
  const long base = (((long)b * Hkv + hk) * Smax + s) * D;
  if (kv == 0) *(uint2*)(kc + base + 32 * (c & 3) + 8 * (c >> 2)) = q;
  else *(uint2*)(vc + base + 8 * c) = q;
  if (c == 0) (kv == 0 ? ksc : vsc)[((long)b * Hkv + hk) * SmaxP + s] = sc;
}

extern "C" int rt_kv_store_fp8(const void* qkv, long ldq, void* kc, void* vc, float* ksc, float* vsc, int B, int S,
                               int Hq, int Hkv, int D, int Smax, int SmaxP, hipStream_t stream) {
  if ((long)B * S == 0) return 0;
  if (D != 128 || S > Smax || SmaxP < Smax || ldq % 8) return -1;
  const long groups = (long)B * S * Hkv * 2;
  hipLaunchKernelGGL(kv_store_fp8_kernel, dim3((unsigned)((groups + 15) / 16)), dim3(256), 0, stream,
                     (const bf16_t*)qkv, ldq, (unsigned char*)kc, (unsigned char*)vc, ksc, vsc, B, S, Hq, Hkv, Smax,
                     SmaxP);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_attn_decode_fused(const void* qkv, long ldq, void* kc, void* vc, int Smax, const int* slot,
                                    const int* attn_len, const int* kv_start, const int* pos, const float* cosT,
                                    const float* sinT, float sign, int window, float* part, unsigned* tickets, int NP,
                                    int PS, void* o, long ldo, int B, int Hq, int Hkv, int D, float scale,
                                    const float* qkv_slabs, int qkv_nsplit, float* ksc, float* vsc, int SmaxP,
                                    long long* stamps, hipStream_t stream) {
  // qkv_slabs: q | k | v given as the qkv GEMM's qkv_nsplit fp32 split-K slabs [nsplit, B, ldq]
  // (summed in the MFMA kernel's prologue; qkv is then unused). ksc / vsc: the caches kc / vc are
  // e4m3fn bytes with per-slot fp32 scales [B, Hkv, SmaxP]. stamps: debug phase stamps or null.
  DecodeFusedArgs a;
  a.qkv = (const bf16_t*)qkv; a.ldq = ldq; a.kc = (bf16_t*)kc; a.vc = (bf16_t*)vc; a.Smax = Smax;
  a.slot = slot; a.attn_len = attn_len; a.kv_start = kv_start; a.pos = pos; a.cosT = cosT; a.sinT = sinT;
  a.sign = sign; a.window = window; a.part = part; a.tickets = tickets; a.o = (bf16_t*)o; a.ldo = ldo;
  a.B = B; a.Hq = Hq; a.Hkv = Hkv; a.NP = NP; a.PS = PS; a.scale_log2 = scale * 1.4426950408889634f;
  a.qkv_slabs = qkv_slabs; a.qkv_nsplit = qkv_slabs ? qkv_nsplit : 0; a.qkv_sstride = (long)B * ldq;
  // K/V cache bytes are read once per decode step: non-temporal loads (batch 256: 56 -> 50 us per
  // layer, profiles/decode_nt_ab.log)
  a.kv_nt = 1;
  a.stamps = stamps;
  a.ksc = ksc; a.vsc = vsc; a.SmaxP = ksc ? SmaxP : 0;
  const bool kv8 = ksc != nullptr;
  if (kv8 && !vsc) return -3;
  if (B == 0) return 0;
  const int G = Hq / Hkv;
  if (G * Hkv != Hq) return -1;
  if (kv8) {
    // fp8 cache: the MFMA kernels only (large batch: one workgroup per (batch, kv head); small
    // batch: 8 waves per (batch, kv head), partitions for long caches)
    if (D != 128 || a.SmaxP < Smax || (G != 1 && G != 2 && G != 4 && G != 8)) return -3;
    // MHA (G = 1) at large batch: the VALU kernel, 2 waves per row (profiles/r3/dec13b_fp8kv_g1_valu_ab.txt)
    if (G == 1 && !a.qkv_slabs && rt_attn_decode_mfma_ok(B, Hq, Hkv, D, NP)) {
      hipLaunchKernelGGL(attn_decode_g1_fp8_kernel<2>, dim3((unsigned)(B * Hkv)), dim3(128), 0, stream, a);
      RT_LAUNCH_CHECK();
      return 0;
    }
    if (rt_attn_decode_mfma_ok(B, Hq, Hkv, D, NP)) {
      dim3 mgrid((unsigned)(B * Hkv)), mblock(64);
      switch (G) {
        case 1: hipLaunchKernelGGL((attn_decode_mfma_kernel<1, 1, true>), mgrid, mblock, 0, stream, a); break;
        case 2: hipLaunchKernelGGL((attn_decode_mfma_kernel<2, 1, true>), mgrid, mblock, 0, stream, a); break;
        case 4: hipLaunchKernelGGL((attn_decode_mfma_kernel<4, 1, true>), mgrid, mblock, 0, stream, a); break;
        default: hipLaunchKernelGGL((attn_decode_mfma_kernel<8, 1, true>), mgrid, mblock, 0, stream, a); break;
      }
    } else {
      if (NP > 1 && !(part && tickets)) return -3;
      const int npm = rt_attn_decode_mw_np(Smax, NP);
      a.NP = npm;
      a.PS = npm > 1 ? ((Smax + npm - 1) / npm + 15) / 16 * 16 : Smax;
      dim3 mgrid((unsigned)(B * Hkv * npm)), mblock(64 * DEC_MW);
      switch (G) {
        case 1: hipLaunchKernelGGL((attn_decode_mfma_kernel<1, DEC_MW, true>), mgrid, mblock, 0, stream, a); break;
        case 2: hipLaunchKernelGGL((attn_decode_mfma_kernel<2, DEC_MW, true>), mgrid, mblock, 0, stream, a); break;
        case 4: hipLaunchKernelGGL((attn_decode_mfma_kernel<4, DEC_MW, true>), mgrid, mblock, 0, stream, a); break;
        default: hipLaunchKernelGGL((attn_decode_mfma_kernel<8, DEC_MW, true>), mgrid, mblock, 0, stream, a); break;
      }
    }
    RT_LAUNCH_CHECK();
    return 0;
  }
  // large batch, one partition per (batch, kv head): the MFMA kernel
  if (rt_attn_decode_mfma_ok(B, Hq, Hkv, D, NP)) {
    dim3 mgrid((unsigned)(B * Hkv)), mblock(64);
    switch (G) {
      case 1: hipLaunchKernelGGL((attn_decode_mfma_kernel<1, 1>), mgrid, mblock, 0, stream, a); break;
      case 2: hipLaunchKernelGGL((attn_decode_mfma_kernel<2, 1>), mgrid, mblock, 0, stream, a); break;
      case 4: hipLaunchKernelGGL((attn_decode_mfma_kernel<4, 1>), mgrid, mblock, 0, stream, a); break;
      case 8: hipLaunchKernelGGL((attn_decode_mfma_kernel<8, 1>), mgrid, mblock, 0, stream, a); break;
      default: hipLaunchKernelGGL((attn_decode_mfma_kernel<16, 1>), mgrid, mblock, 0, stream, a); break;
    }
    RT_LAUNCH_CHECK();
    return 0;
  }
  // small batch, short caches: 8 waves per (batch, kv head), merged in LDS
  if (rt_attn_decode_mw_ok(B, Hq, Hkv, D, Smax) && !a.qkv_slabs && (NP <= 1 || (part && tickets))) {
    const int npm = rt_attn_decode_mw_np(Smax, NP);
    a.NP = npm;
    a.PS = npm > 1 ? ((Smax + npm - 1) / npm + 15) / 16 * 16 : Smax;
    // 8 waves per (row, kv head) up to 256 pairs (one 512-thread workgroup per CU); 4 waves above
    // (serving at batch 32..127: 1024-2048 waves instead of one chain of tiles per pair)
    const bool w4 = (long)B * Hkv >= 256;
    dim3 mgrid((unsigned)(B * Hkv * npm)), mblock(64 * (w4 ? 4 : DEC_MW));
    if (w4) {
      switch (G) {
        case 1: hipLaunchKernelGGL((attn_decode_mfma_kernel<1, 4>), mgrid, mblock, 0, stream, a); break;
        case 2: hipLaunchKernelGGL((attn_decode_mfma_kernel<2, 4>), mgrid, mblock, 0, stream, a); break;
        case 4: hipLaunchKernelGGL((attn_decode_mfma_kernel<4, 4>), mgrid, mblock, 0, stream, a); break;
        default: hipLaunchKernelGGL((attn_decode_mfma_kernel<8, 4>), mgrid, mblock, 0, stream, a); break;
      }
    } else {
      switch (G) {
        case 1: hipLaunchKernelGGL((attn_decode_mfma_kernel<1, DEC_MW>), mgrid, mblock, 0, stream, a); break;
        case 2: hipLaunchKernelGGL((attn_decode_mfma_kernel<2, DEC_MW>), mgrid, mblock, 0, stream, a); break;
        case 4: hipLaunchKernelGGL((attn_decode_mfma_kernel<4, DEC_MW>), mgrid, mblock, 0, stream, a); break;
        default: hipLaunchKernelGGL((attn_decode_mfma_kernel<8, DEC_MW>), mgrid, mblock, 0, stream, a); break;
      }
    }
    RT_LAUNCH_CHECK();
    return 0;
  }
  if (a.qkv_slabs) return -2;  // the slab form exists only in the MFMA kernel (caller reduces first)
  const int nk = 4;  // keys per lane per chunk; PS must be a multiple of the chunk
  if (PS % (4 * (64 / (D / 8)) * nk) != 0) return -1;
  dim3 grid(NP, Hkv, B), block(256);
#define DF_CASE(DD, GG, NN)                                                                   \
  if (D == DD && G == GG && nk == NN) {                                                       \
    hipLaunchKernelGGL((attn_decode_fused_kernel<DD, GG, NN>), grid, block, 0, stream, a);    \
    RT_LAUNCH_CHECK();                                                                        \
    return 0;                                                                                 \
  }
#define DF_G(DD, NN) DF_CASE(DD, 1, NN) DF_CASE(DD, 2, NN) DF_CASE(DD, 4, NN) DF_CASE(DD, 8, NN)
  DF_G(128, 4) DF_G(64, 4) DF_G(32, 4)
#undef DF_G
#undef DF_CASE
  return -1;
}

extern "C" int rt_rope_qkv(void* qkv, long ld, const int* pos, const float* cosT, const float* sinT, int T, int S,
                           int Hq, int Hkv, int D, float sign, void* kc, void* vc, const int* slot_base, int Smax,
                           int do_rope_q, hipStream_t stream);

// rope_pos / rope_cos / rope_sin (all or none): the RoPE backward of the forward's q / k rotation,
// fused into the dQ / dK stores. dq_f32: unused (kept in the signature; dQ is written in bf16 by
// attn_bwd_dq_kernel, no fp32 accumulator).
extern "C" int rt_attn_bwd(const void* q, long ldq, const void* k, long ldk, const void* v, long ldv, const void* o,
                           long ldo, const void* dout, long lddo, const float* lse, float* delta, float* dq_f32,
                           void* dq, long lddq, void* dk, long lddk, void* dv, long lddv, const int* kv_start, int B,
                           int S, int Hq, int Hkv, int D, int causal, int window, float scale, const int* rope_pos,
                           const float* rope_cos, const float* rope_sin, hipStream_t stream) {
  AttnBwdArgs a;
  a.q = (const bf16_t*)q; a.ldq = ldq; a.k = (const bf16_t*)k; a.ldk = ldk; a.v = (const bf16_t*)v; a.ldv = ldv;
  a.o = (const bf16_t*)o; a.ldo = ldo; a.dout = (const bf16_t*)dout; a.lddo = lddo; a.lse = lse; a.delta = delta;
  a.dq = dq_f32; a.dk = (bf16_t*)dk; a.lddk = lddk; a.dv = (bf16_t*)dv; a.lddv = lddv; a.kv_start = kv_start;
  a.B = B; a.S = S; a.Hq = Hq; a.Hkv = Hkv; a.causal = causal; a.window = window;
  a.scale = scale; a.scale_log2 = scale * 1.4426950408889634f;
  a.lpt = 0;
  if ((rope_pos != nullptr) != (rope_cos != nullptr) || (rope_cos != nullptr) != (rope_sin != nullptr)) return -2;
  a.rope_pos = rope_pos; a.rope_cos = rope_cos; a.rope_sin = rope_sin;
  if (B == 0 || S == 0) return 0;
  a.dqb = (bf16_t*)dq; a.lddq = lddq;
  const long rows = (long)B * S * Hq;
  const long rows_per_block = 4L * (64 / (D / 8));
  dim3 pgrid((unsigned)((rows + rows_per_block - 1) / rows_per_block)), grid((S + 63) / 64, Hkv, B);
  // dK / dV per 64-key block, dQ by a separate kernel per 64-query block (no atomics)
  if (D != 64 && D != 128) return -1;
  // GQA-4, causal, short sequences: dQ on head-packed 16-position workgroups
  const bool dq_hp = D == 128 && Hkv * 4 == Hq && causal && S <= tuning().attn_dq_hp_maxs;
  dim3 qgrid = dq_hp ? dim3((S + 15) / 16, Hkv, B) : dim3((S + 63) / 64, Hq, B);
#define BWD_CASE(DD)                                                                              \
  hipLaunchKernelGGL(attn_bwd_pre_kernel<DD>, pgrid, dim3(256), 0, stream, a);                    \
  hipLaunchKernelGGL(attn_bwd_kernel<DD>, grid, dim3(256), 0, stream, a);
  a.lpt = attn_lpt_on(grid, causal);
  if (D == 64) { BWD_CASE(64) } else { BWD_CASE(128) }
#undef BWD_CASE
  a.lpt = attn_lpt_on(qgrid, causal);
  if (D == 64) hipLaunchKernelGGL((attn_bwd_dq_kernel<64>), qgrid, dim3(256), 0, stream, a);
  else if (dq_hp) hipLaunchKernelGGL((attn_bwd_dq_kernel<128, true>), qgrid, dim3(256), 0, stream, a);
  else hipLaunchKernelGGL((attn_bwd_dq_kernel<128>), qgrid, dim3(256), 0, stream, a);
  RT_LAUNCH_CHECK();
  return 0;
}



