// g2v_coexpr.hip -- gene co-expression pairs on the GPU.
//
// Replaces the per-study hot loop of src/generate_gene_pairs.py:45-65 (coexpr):
//
//     corr = data.corr().abs()                       # pandas Pearson, fp64
//     rows, cols = (corr > corr_threshold).values.nonzero()
//     pairs = [(r, c) for r, c in zip(rows, cols) if r != c]
//
// data is [samples][genes].  pandas computes G^2/2 Welford correlations in a
// Cython loop (O(G^2 n), minutes to hours at 20k-60k genes); here:
//
//   k_coexpr_stats   one thread per gene: fp64 mean, centred sum of squares,
//                    constant-column flag; writes z[k][g] = (x - mean) / sqrt(M2)
//                    so that corr(g, h) = sum_k z[k][g] z[k][h]
//   k_coexpr_mask_mfma  64 x 64 gene tile per workgroup (upper triangle only,
//                    off-diagonal tiles also write their transposed bits), four
//                    32 x 32 wave tiles of v_mfma_f64_16x16x4_f64, K (samples)
//                    staged through LDS 16 at a time (next stage prefetched into
//                    registers during the MFMAs); the epilogue never writes
//                    the G x G matrix, only a bit per (row, col): |r| > threshold,
//                    r != c, neither column constant (pandas: NaN, never > t)
//   k_coexpr_count   popcount per row
//   k_coexpr_scan    exclusive scan of the row counts (one workgroup)
//   k_coexpr_emit    one wave per row: (row, col) int32 pairs in nonzero()
//                    order (row-major, columns ascending)
//
// fp64 throughout: gfx950's fp64 MFMA rate equals its fp64 vector rate, and
// fp64 keeps |r| within ~1e-15 of pandas' Welford value, so
// the pair SET equals pandas' except for |r| within that distance of the
// threshold (the parity tests assert none exist in their fixtures).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <string>

#include "g2v.h"
#include "g2v_internal.h"

namespace {

constexpr int kTile = 64;   // genes per tile side
constexpr int kKt = 16;     // samples per LDS stage

__global__ void k_coexpr_stats(const double* __restrict__ x, int64_t n, int64_t G, int64_t gp,
                               double* __restrict__ z, uint8_t* __restrict__ cst) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  double s = 0.0, lo = x[g], hi = x[g];
  for (int64_t k = 0; k < n; ++k) {
    const double v = x[k * G + g];
    s += v;
    lo = v < lo ? v : lo;
    hi = v > hi ? v : hi;
  }
  const double mean = s / (double)n;
  double m2 = 0.0;
  for (int64_t k = 0; k < n; ++k) {
    const double d = x[k * G + g] - mean;
    m2 = fma(d, d, m2);
  }
  const bool constant = !(hi > lo) || !(m2 > 0.0);
  cst[g] = constant ? 1 : 0;
  const double inv = constant ? 0.0 : 1.0 / sqrt(m2);
  for (int64_t k = 0; k < n; ++k) z[k * gp + g] = (x[k * G + g] - mean) * inv;
}

// The correlation tile on the matrix cores: v_mfma_f64_16x16x4_f64 (gfx950:
// fp64 matrix rate == fp64 vector rate; an MFMA takes 2 operand doubles per
// lane for 16 FMAs per lane).  64 x 64 genes per workgroup, wave w owns the
// 32 x 32 sub-tile (rows 32*(w>>1), cols 32*(w&1)) as 2 x 2 MFMA blocks.
// Measured at 20k genes x 100 samples: 1.18 ms (38 TF/s of issued fp64 FMA,
// 48 % of peak) with the next stage prefetched into registers; 1.34 ms without
// the prefetch (the same as a 4 x 4 fp64 VALU register tile), 1.83 ms with
// 128 x 128 tiles, 1.38 ms with 32-sample stages (padding n to 32): the tile is
// bound by the per-stage z-load latency, not by the FMA pipe.  Operand maps
// (cdna_hip_programming.md, f64 form): A[r = l&15][k = l>>4],
// B[k = l>>4][c = l&15]; D reg q: row (l>>4) + 4q, col l&15.
typedef double d4_t __attribute__((ext_vector_type(4)));

// LDS row pitch in doubles: rows k and k+1 of a stage land 32 banks apart, so
// the 32 lanes of each half of a ds_read_b64 (16 genes x 2 samples) hit 64
// distinct banks
constexpr int kLds = kTile + 16;

// Block b -> upper-triangle tile (ty, tx), tx >= ty, of a words x words tile
// grid.  Workgroups are dealt to the 8 XCDs round-robin, so block b runs on
// XCD b % 8; each XCD gets one contiguous run of row-major tiles, and the row
// panels those tiles share stay in that XCD's L2.  False for padding blocks.
__device__ inline bool tri_tile(int64_t b, int64_t nblocks, int64_t words, int64_t* ty,
                                int64_t* tx) {
  const int64_t T = words * (words + 1) / 2;
  const int64_t per = nblocks / 8;  // nblocks is a multiple of 8
  const int64_t l = (b % 8) * per + b / 8;
  if (l >= T) return false;
  // row y starts at s(y) = y*words - y*(y-1)/2; invert with sqrt, then fix up
  const double wd = 2.0 * (double)words + 1.0;
  int64_t y = (int64_t)((wd - sqrt(wd * wd - 8.0 * (double)l)) * 0.5);
  if (y < 0) y = 0;
  if (y >= words) y = words - 1;
  auto start = [words](int64_t r) { return r * words - r * (r - 1) / 2; };
  while (y > 0 && start(y) > l) --y;
  while (y + 1 < words && start(y + 1) <= l) ++y;
  *ty = y;
  *tx = y + (l - start(y));
  return true;
}

__global__ __launch_bounds__(256) void k_coexpr_mask_mfma(const double* __restrict__ z,
                                                          int64_t npad, int64_t gp, int64_t G,
                                                          const uint8_t* __restrict__ cst,
                                                          double thr,
                                                          uint64_t* __restrict__ mask) {
  __shared__ double sa[kKt][kLds];
  __shared__ double sb[kKt][kLds];
  __shared__ unsigned long long sm[kTile];
  __shared__ unsigned long long smt[kTile];
  // symmetric: only the upper-triangle tiles are launched, XCD-contiguous
  int64_t ty, tx;
  if (!tri_tile(blockIdx.x, gridDim.x, gp / kTile, &ty, &tx)) return;
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  const int wr = (w >> 1) * 32, wc = (w & 1) * 32;
  const int64_t r0 = ty * kTile, c0 = tx * kTile;
  if (t < kTile) {
    sm[t] = 0ull;
    smt[t] = 0ull;
  }
  d4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = d4_t{0.0, 0.0, 0.0, 0.0};
  const int fr = lane & 15, fk = lane >> 4;
  // 16 x 64 doubles per operand and stage, 4 per thread, coalesced along genes;
  // the next stage's loads are in flight while this stage's MFMAs run
  double pa[4], pb[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int idx = q * 256 + t;
    pa[q] = z[(int64_t)(idx >> 6) * gp + r0 + (idx & 63)];
    pb[q] = z[(int64_t)(idx >> 6) * gp + c0 + (idx & 63)];
  }
  for (int64_t k0 = 0; k0 < npad; k0 += kKt) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = q * 256 + t;
      sa[idx >> 6][idx & 63] = pa[q];
      sb[idx >> 6][idx & 63] = pb[q];
    }
    __syncthreads();
    if (k0 + kKt < npad) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int idx = q * 256 + t;
        pa[q] = z[(k0 + kKt + (idx >> 6)) * gp + r0 + (idx & 63)];
        pb[q] = z[(k0 + kKt + (idx >> 6)) * gp + c0 + (idx & 63)];
      }
    }
#pragma unroll
    for (int ks = 0; ks < kKt; ks += 4) {
      double a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[i] = sa[ks + fk][wr + 16 * i + fr];
        b[i] = sb[ks + fk][wc + 16 * i + fr];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // one bit per (row, col) and, off the diagonal, per (col, row).  A constant
  // column has z == 0, so its r is exactly 0 and never > thr >= 0: the flags
  // are only read for a negative threshold.
  const bool offdiag = tx != ty;
  const bool chk = thr < 0.0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rl = wr + 16 * i + fk + 4 * q;
        const int cl = wc + 16 * j + fr;
        const int64_t r = r0 + rl, c = c0 + cl;
        const bool on = r < G && c < G && r != c && fabs(acc[i][j][q]) > thr &&
                        !(chk && (cst[r] || cst[c]));
        if (on) {
          atomicOr(&sm[rl], 1ull << cl);
          if (offdiag) atomicOr(&smt[cl], 1ull << rl);
        }
      }
  __syncthreads();
  if (t < kTile) {
    mask[(r0 + t) * (gp / kTile) + tx] = sm[t];
    if (offdiag) mask[(c0 + t) * (gp / kTile) + ty] = smt[t];
  }
}

__global__ void k_coexpr_count(const uint64_t* __restrict__ mask, int64_t gp,
                               int64_t* __restrict__ cnt) {
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= gp) return;
  const int64_t words = gp / kTile;
  int64_t c = 0;
  for (int64_t w = lane; w < words; w += 64) c += __popcll(mask[r * words + w]);
  for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m, 64);
  if (lane == 0) cnt[r] = c;
}

// exclusive scan of cnt[0..n) into off[0..n], off[n] = total (one workgroup)
__global__ __launch_bounds__(1024) void k_coexpr_scan(const int64_t* __restrict__ cnt, int64_t n,
                                                      int64_t* __restrict__ off) {
  __shared__ int64_t sw[16];
  __shared__ int64_t carry;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  if (t == 0) carry = 0;
  __syncthreads();
  for (int64_t b = 0; b < n; b += 1024) {
    const int64_t i = b + t;
    const int64_t v = i < n ? cnt[i] : 0;
    int64_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) sw[wid] = x;
    __syncthreads();
    int64_t base = carry;
    for (int w = 0; w < wid; ++w) base += sw[w];
    if (i < n) off[i] = base + x - v;
    __syncthreads();
    if (t == 1023) carry = base + x;
    __syncthreads();
  }
  if (t == 0) off[n] = carry;
}

// one wave per row: lanes own mask words, a wave prefix sum orders them
__global__ void k_coexpr_emit(const uint64_t* __restrict__ mask, int64_t gp, int64_t G,
                              const int64_t* __restrict__ off, int32_t* __restrict__ pairs) {
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= G) return;
  const int64_t words = gp / kTile;
  int64_t pos = off[r];
  for (int64_t w0 = 0; w0 < words; w0 += 64) {
    const int64_t w = w0 + lane;
    uint64_t m = w < words ? mask[r * words + w] : 0ull;
    const int64_t c = __popcll(m);
    int64_t x = c;
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    int64_t p = pos + x - c;
    while (m) {
      const int b = __builtin_ctzll(m);
      m &= m - 1;
      pairs[2 * p] = (int32_t)r;
      pairs[2 * p + 1] = (int32_t)(w * kTile + b);
      ++p;
    }
    pos += __shfl(x, 63, 64);
  }
}

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

// device timings of the calling thread's last g2v_coexpr_pairs call (ms)
thread_local double t_mask_ms = 0.0, t_total_ms = 0.0;

struct Events {
  hipEvent_t e[4] = {nullptr, nullptr, nullptr, nullptr};
  ~Events() {
    for (hipEvent_t x : e)
      if (x) (void)hipEventDestroy(x);
  }
};

}  // namespace

#define CX_CHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      rc = g2v::set_error(G2V_EHIP, std::string(#x) + " failed: " + hipGetErrorString(e_)); \
      goto done;                                                                    \
    }                                                                               \
  } while (0)

extern "C" int g2v_coexpr_pairs(int device, const double* x, int64_t n_samples, int64_t n_genes,
                                double threshold, int32_t* pairs, int64_t cap,
                                int64_t* n_pairs) {
  if (!x || !n_pairs || n_samples < 1 || n_genes < 0 || (pairs == nullptr && cap != 0) ||
      cap < 0 || n_genes > (int64_t)INT32_MAX) {
    return g2v::set_error(G2V_EINVAL, "g2v_coexpr_pairs: bad arguments");
  }
  *n_pairs = 0;
  if (n_genes == 0) return G2V_OK;
  int rc = G2V_OK;
  const int64_t G = n_genes, n = n_samples;
  const int64_t gp = (G + kTile - 1) / kTile * kTile;
  const int64_t npad = (n + kKt - 1) / kKt * kKt;
  const int64_t words = gp / kTile;
  // one workspace allocation, carved into 256-B aligned pieces
  auto al = [](int64_t b) { return (b + 255) / 256 * 256; };
  const int64_t o_x = 0, o_z = o_x + al(8 * n * G), o_m = o_z + al(8 * npad * gp),
                o_n = o_m + al(8 * gp * words), o_off = o_n + al(8 * gp),
                o_c = o_off + al(8 * (gp + 1)), ws_bytes = o_c + al(G);
  DevBuf ws, dp;
  Events ev;
  hipStream_t st = nullptr;
  int64_t total = 0;
  float ms = 0.f;
  t_mask_ms = t_total_ms = 0.0;
  CX_CHK(hipSetDevice(device));
  CX_CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  for (hipEvent_t& e : ev.e) CX_CHK(hipEventCreate(&e));
  CX_CHK(hipMalloc(&ws.p, (size_t)ws_bytes));
  CX_CHK(hipEventRecord(ev.e[0], st));
  {
    char* base = (char*)ws.p;
    double* dx = (double*)(base + o_x);
    double* dz = (double*)(base + o_z);
    uint64_t* dm = (uint64_t*)(base + o_m);
    int64_t* dn = (int64_t*)(base + o_n);
    int64_t* doff = (int64_t*)(base + o_off);
    uint8_t* dc = (uint8_t*)(base + o_c);
    CX_CHK(hipMemcpyAsync(dx, x, sizeof(double) * n * G, hipMemcpyHostToDevice, st));
    CX_CHK(hipMemsetAsync(dz, 0, sizeof(double) * npad * gp, st));
    hipLaunchKernelGGL(k_coexpr_stats, dim3((unsigned)((G + 255) / 256)), dim3(256), 0, st,
                       (const double*)dx, n, G, gp, dz, dc);
    CX_CHK(hipGetLastError());
    CX_CHK(hipEventRecord(ev.e[1], st));
    const int64_t tiles = words * (words + 1) / 2;
    hipLaunchKernelGGL(k_coexpr_mask_mfma, dim3((unsigned)((tiles + 7) / 8 * 8)), dim3(256), 0,
                       st, (const double*)dz, npad, gp, G, (const uint8_t*)dc, threshold, dm);
    CX_CHK(hipGetLastError());
    CX_CHK(hipEventRecord(ev.e[2], st));
    hipLaunchKernelGGL(k_coexpr_count, dim3((unsigned)((gp + 3) / 4)), dim3(256), 0, st,
                       (const uint64_t*)dm, gp, dn);
    CX_CHK(hipGetLastError());
    hipLaunchKernelGGL(k_coexpr_scan, dim3(1), dim3(1024), 0, st, (const int64_t*)dn, G, doff);
    CX_CHK(hipGetLastError());
    CX_CHK(hipMemcpyAsync(&total, doff + G, sizeof total, hipMemcpyDeviceToHost, st));
    CX_CHK(hipStreamSynchronize(st));
  }
  *n_pairs = total;
  if (pairs && total > 0 && cap >= total) {
    CX_CHK(hipMalloc(&dp.p, sizeof(int32_t) * 2 * total));
    char* base = (char*)ws.p;
    hipLaunchKernelGGL(k_coexpr_emit, dim3((unsigned)((G + 3) / 4)), dim3(256), 0, st,
                       (const uint64_t*)(base + o_m), gp, G, (const int64_t*)(base + o_off),
                       (int32_t*)dp.p);
    CX_CHK(hipGetLastError());
    CX_CHK(hipMemcpyAsync(pairs, dp.p, sizeof(int32_t) * 2 * total, hipMemcpyDeviceToHost, st));
    CX_CHK(hipStreamSynchronize(st));
  } else if (pairs && cap < total) {
    rc = g2v::set_error(G2V_ERANGE, "g2v_coexpr_pairs: capacity " + std::to_string(cap) + " < " +
                                        std::to_string(total) + " pairs (*n_pairs holds the count)");
  }
  CX_CHK(hipEventRecord(ev.e[3], st));
  CX_CHK(hipEventSynchronize(ev.e[3]));
  CX_CHK(hipEventElapsedTime(&ms, ev.e[1], ev.e[2]));
  t_mask_ms = ms;
  CX_CHK(hipEventElapsedTime(&ms, ev.e[0], ev.e[3]));
  t_total_ms = ms;
done:
  if (st) (void)hipStreamDestroy(st);
  return rc;
}

extern "C" int g2v_coexpr_last_timing(double* mask_ms, double* total_ms) {
  if (!mask_ms || !total_ms) return g2v::set_error(G2V_EINVAL, "g2v_coexpr_last_timing: null output");
  *mask_ms = t_mask_ms;
  *total_ms = t_total_ms;
  return G2V_OK;
}
