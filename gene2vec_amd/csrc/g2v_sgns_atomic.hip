// g2v_sgns_atomic.hip -- k_sgns_atomic: the production Hogwild SGNS kernel
// (memory-side float atomics, hot-row stripes).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "g2v_internal.h"
#include "g2v_device.h"

namespace g2v {

// ---------------------------------------------------------------------------
// k_sgns_atomic: the production Hogwild kernel
// ---------------------------------------------------------------------------
// Same per-example math as k_sgns, but every table update is a memory-side
// float atomic of the delta (g * syn0[input] into syn1neg[t], lockf * work
// into syn0[input]).  With ~4k examples in flight on 256 CUs every row of a
// 24k-gene vocabulary is touched every few microseconds, so plain
// read-modify-write stores lose most updates (measured: iteration-0 loss 4.15
// vs 2.77 sequential); atomics keep all of them (2.76).
//
// Pipelining: example e+1's record and rows are loaded BEFORE example e's
// atomics are issued, so in the wave's in-order vmcnt they wait only behind
// example e-1's atomics (the record load's wait drains those; a wave keeps at
// most one example's atomics in flight).  l1 and work are staged through LDS in element order
// so each atomic wave-instruction adds 64 contiguous floats (256 B); the
// D % 64 tails of all K+2 rows are packed into shared instructions.
template <int K, int NV>
struct ExRegs {
  int32_t tg[K + 1];
  int32_t input;
  float alpha;
  float4 l1[NV];
  float4 rw[K + 1][NV];
};

// row t of table tbl (0 = syn0, 1 = syn1neg) as this lane's float4 column(s):
// main row plus its stripe copies when t is a striped hot row
template <int NV>
__device__ __forceinline__ void load_row(float4 (&o)[NV], const SgnsArgs& a,
                                         __amdgpu_buffer_rsrc_t rmain, int t, int tbl, int rowb,
                                         int lane, const bool (&on)[NV]) {
  const int off = t * rowb + lane * 16;
#pragma unroll
  for (int v = 0; v < NV; ++v)
    o[v] = on[v] ? bload4<0>(rmain, off + 1024 * v) : make_float4(0.f, 0.f, 0.f, 0.f);
  if (t < a.stripe_rows) {
    const float* sb = a.stripe + (int64_t)tbl * (a.stripe_copies - 1) * a.stripe_rows * a.ld;
    for (int c = 1; c < a.stripe_copies; ++c) {
      const float4* sr = reinterpret_cast<const float4*>(
          sb + ((int64_t)(c - 1) * a.stripe_rows + t) * a.ld);
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        if (!on[v]) continue;
        const float4 q = sr[lane + 64 * v];
        o[v].x += q.x;
        o[v].y += q.y;
        o[v].z += q.z;
        o[v].w += q.w;
      }
    }
  }
}

// destination of an atomic delta for row t of table tbl: main or stripe copy c
// (WR 4, ablation: the same rows of a scratch table the kernel never reads)
template <int WR = 0>
__device__ __forceinline__ float* upd_row(const SgnsArgs& a, int tbl, int t, int c) {
  if (WR == 4) {
    const int64_t nrow = (int64_t)a.V + (int64_t)(a.stripe_copies - 1) * a.stripe_rows;
    const int64_t rr =
        (c == 0 || t >= a.stripe_rows) ? t : a.V + (int64_t)(c - 1) * a.stripe_rows + t;
    return reinterpret_cast<float*>(a.dbg16) + (tbl * nrow + rr) * a.ld;
  }
  if (c == 0 || t >= a.stripe_rows) return (tbl ? a.wr1 : a.wr0) + (int64_t)t * a.ld;
  return a.stripe + (((int64_t)tbl * (a.stripe_copies - 1) + (c - 1)) * a.stripe_rows + t) * a.ld;
}

template <int K, int NV>
__device__ __forceinline__ void load_example(ExRegs<K, NV>& x, const SgnsArgs& a, int64_t e,
                                             __amdgpu_buffer_rsrc_t r0,
                                             __amdgpu_buffer_rsrc_t r1, int rowb, int lane,
                                             const bool (&on)[NV]) {
  const int32_t* r = a.rec + e * a.rec_stride;
  x.tg[0] = __builtin_amdgcn_readfirstlane(r[0]);
  x.input = __builtin_amdgcn_readfirstlane(r[1]);
  x.alpha = __int_as_float(__builtin_amdgcn_readfirstlane(r[2]));
#pragma unroll
  for (int d = 0; d < K; ++d) x.tg[d + 1] = __builtin_amdgcn_readfirstlane(r[3 + d]);
  load_row<NV>(x.l1, a, r0, x.input, 0, rowb, lane, on);
#pragma unroll
  for (int d = 0; d <= K; ++d) {
    if (x.tg[d] >= 0) {
      load_row<NV>(x.rw[d], a, r1, x.tg[d], 1, rowb, lane, on);
    } else {
#pragma unroll
      for (int v = 0; v < NV; ++v) x.rw[d][v] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

// WR (debug ablation only): 0 atomics (production), 1 same-shape plain stores,
// 2 no table writes, 3 packed-f16 atomics into a scratch table (half the atomic
// bytes, tables never written: a throughput probe), 4 the production f32
// atomics into that scratch table (tables never written), 5 production atomics
// on syn1neg only, syn0 never written (the ceiling of any syn0-side combining)
template <int WR>
__device__ __forceinline__ void upd(float* p, float v) {
  if (WR == 0 || WR == 4 || WR == 5) atomicAdd(p, v);
  else if (WR == 1) *p = v;
}

// LOSS ([ext] compute_loss): each wave keeps a float32 partial of the
// -log(sigmoid(+-f)) LOG_TABLE terms over its chunk and adds it to a double
// accumulator once per chunk; LOSS = false compiles the tally out.
template <int K, int NV, int WR = 0, bool LOSS = false>
__global__ __launch_bounds__(kSgnsThreads) void k_sgns_atomic(SgnsArgs a) {
  constexpr int NT = K + 1;
  constexpr int W = kSgnsThreads / 64;
  __shared__ float s_lut[kExpTableSize];
  __shared__ float s_log[LOSS ? kExpTableSize : 1];
  __shared__ float s_l1[W][256 * NV];
  __shared__ float s_wk[W][256 * NV];
  for (int i = threadIdx.x; i < kExpTableSize; i += kSgnsThreads) {
    s_lut[i] = a.exp_table[i];
    if (LOSS) s_log[i] = a.log_table[i];
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int64_t gw = (int64_t)blockIdx.x * W + wid;
  const int64_t nw = (int64_t)gridDim.x * W;
  const int64_t E = *a.n_examples;
  const int D = a.D;
  const int full = D >> 6;           // whole 64-float atomic groups per row
  const int tail = D & 63;           // leftover floats per row
  const int tpack = tail ? 64 / tail : 0;  // row tails per packed instruction
  const int64_t tbytes = (int64_t)a.V * a.ld * 4;
  const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.rd0, tbytes);
  const __amdgpu_buffer_rsrc_t r1 = make_rsrc(a.rd1, tbytes);
  const int rowb = (int)a.ld * 4;
  float* s1 = s_l1[wid];
  float* sw = s_wk[wid];
  bool on[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) on[v] = (lane + 64 * v) < a.nvec;

  for (int64_t c = gw; c * kChunk < E; c += nw) {
    const int64_t e_beg = c * kChunk;
    const int64_t e_end = (e_beg + kChunk < E) ? e_beg + kChunk : E;
    float lsum = 0.f;
    ExRegs<K, NV> x;
    load_example<K, NV>(x, a, e_beg, r0, r1, rowb, lane, on);
    for (int64_t e = e_beg; e < e_end; ++e) {
      // ---- compute example e ------------------------------------------------
      double pd[NT], dot[NT];
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        double s = 0.0;
#pragma unroll
        for (int v = 0; v < NV; ++v) s = dot4(x.l1[v], x.rw[d][v], s);
        pd[d] = s;
      }
      wave_reduce_multi<NT>(pd, dot, lane);
      float4 work[NV];
#pragma unroll
      for (int v = 0; v < NV; ++v) work[v] = make_float4(0.f, 0.f, 0.f, 0.f);
      float g[NT];
      bool dirty[NT];
      bool any = false;
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        g[d] = 0.f;
        dirty[d] = false;
        if (x.tg[d] < 0) continue;
        double dt = dot[d];
        bool prev_dirty = false;
#pragma unroll
        for (int d2 = 0; d2 < d; ++d2) {
          if (x.tg[d2] == x.tg[d]) {
#pragma unroll
            for (int v = 0; v < NV; ++v) x.rw[d][v] = x.rw[d2][v];
            prev_dirty = dirty[d2];
          }
        }
        if (prev_dirty) {
          double s = 0.0;
#pragma unroll
          for (int v = 0; v < NV; ++v) s = dot4(x.l1[v], x.rw[d][v], s);
          dt = wave_allreduce_d(s);
          dirty[d] = true;
        }
        const float f = (float)dt;
        if (f <= -(float)kMaxExp || f >= (float)kMaxExp) continue;
        const int idx = (int)((f + (float)kMaxExp) * (float)kLutScale);
        const float gg = ((d == 0 ? 1.0f : 0.0f) - s_lut[idx]) * x.alpha;
        if (LOSS) {
          const float fl = d == 0 ? f : -f;
          lsum = lsum - s_log[(int)((fl + (float)kMaxExp) * (float)kLutScale)];
        }
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          work[v].x = __fmaf_rn(gg, x.rw[d][v].x, work[v].x);
          work[v].y = __fmaf_rn(gg, x.rw[d][v].y, work[v].y);
          work[v].z = __fmaf_rn(gg, x.rw[d][v].z, work[v].z);
          work[v].w = __fmaf_rn(gg, x.rw[d][v].w, work[v].w);
          x.rw[d][v].x = __fmaf_rn(gg, x.l1[v].x, x.rw[d][v].x);
          x.rw[d][v].y = __fmaf_rn(gg, x.l1[v].y, x.rw[d][v].y);
          x.rw[d][v].z = __fmaf_rn(gg, x.l1[v].z, x.rw[d][v].z);
          x.rw[d][v].w = __fmaf_rn(gg, x.l1[v].w, x.rw[d][v].w);
        }
        g[d] = gg;
        dirty[d] = true;
        any = true;
      }
      // stage l1 / work in element order
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        *reinterpret_cast<float4*>(s1 + (lane + 64 * v) * 4) = x.l1[v];
        *reinterpret_cast<float4*>(sw + (lane + 64 * v) * 4) = work[v];
      }
      __builtin_amdgcn_wave_barrier();
      int32_t tg[NT];
#pragma unroll
      for (int d = 0; d < NT; ++d) tg[d] = x.tg[d];
      const int32_t input = x.input;
      const float lf = any ? a.lockf[input] : 0.f;

      // ---- prefetch example e+1 (its loads overtake e's atomics) -------------
      if (e + 1 < e_end) load_example<K, NV>(x, a, e + 1, r0, r1, rowb, lane, on);

      // ---- atomics of example e -----------------------------------------------
      const int cbase = (int)(e % (int64_t)a.stripe_copies);
      if (WR == 3) {
        typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
        const int hw = (int)(a.ld >> 1);
        const int n2 = (D + 1) >> 1;  // half2 words per row
        const int64_t nrow = (int64_t)a.V + (int64_t)(a.stripe_copies - 1) * a.stripe_rows;
#pragma unroll
        for (int d = 0; d <= NT; ++d) {
          const bool w = d == NT;
          const float cf = w ? (any ? lf : 0.f) : g[d];
          if (cf == 0.f) continue;
          const int t = w ? input : tg[d];
          // hot rows keep their stripe copies: copy c of row t lives at V + (c-1)*rows + t
          const int cc = (cbase + d) % a.stripe_copies;
          const int64_t rr = (cc == 0 || t >= a.stripe_rows)
                                 ? t : a.V + (int64_t)(cc - 1) * a.stripe_rows + t;
          uint32_t* row = a.dbg16 + ((w ? 0 : 1) * nrow + rr) * hw;
          const float* src = w ? sw : s1;
          for (int i = lane; i < n2; i += 64) {
            h2_t v;
            v.x = (_Float16)(cf * src[2 * i]);
            v.y = (_Float16)(cf * src[2 * i + 1]);
            __builtin_amdgcn_global_atomic_fadd_v2f16(reinterpret_cast<h2_t*>(row + i), v);
          }
        }
        __builtin_amdgcn_wave_barrier();
        continue;
      }
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        if (g[d] == 0.f) continue;
        float* row = upd_row<WR>(a, 1, tg[d], (cbase + d) % a.stripe_copies) + lane;
        for (int i = 0; i < full; ++i) upd<WR>(row + 64 * i, g[d] * s1[64 * i + lane]);
      }
      if (any && WR != 5) {
        float* row = upd_row<WR>(a, 0, input, (cbase + NT) % a.stripe_copies) + lane;
        for (int i = 0; i < full; ++i) upd<WR>(row + 64 * i, lf * sw[64 * i + lane]);
      }
      if (tail && any) {
        // rows q = 0..K: syn1neg[tg[q]] += g[q] * l1; q = K+1: syn0[input] += lf * work
        for (int q0 = 0; q0 < NT + 1; q0 += tpack) {
          const int q = q0 + lane / tail;
          const int el = full * 64 + lane % tail;
          float coef = 0.f;
          int row_t = 0;
#pragma unroll
          for (int d = 0; d < NT; ++d) {
            if (q == d) {
              coef = g[d];
              row_t = tg[d] < 0 ? 0 : tg[d];
            }
          }
          const bool from_work = (q == NT);
          if (from_work) {
            coef = (any && WR != 5) ? lf : 0.f;
            row_t = input;
          }
          if (lane / tail < tpack && q <= NT && coef != 0.f) {
            const float src = from_work ? sw[el] : s1[el];
            float* row = upd_row<WR>(a, from_work ? 0 : 1, row_t, (cbase + q) % a.stripe_copies);
            upd<WR>(row + el, coef * src);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (LOSS && lane == 0 && lsum != 0.f) atomicAdd(a.loss_f64, (double)lsum);
  }
}


#ifndef G2V_K
#error "g2v_sgns_atomic.hip is compiled once per negative count: -DG2V_K=<K>"
#endif
#define G2V_CAT2(a, b) a##b
#define G2V_CAT(a, b) G2V_CAT2(a, b)

hipError_t G2V_CAT(launch_sgns_atomic_k, G2V_K)(const SgnsArgs& a, int nv, int grid,
                                                 hipStream_t st) {
#if G2V_K == 5
  // ablation builds (G2V_OPT_DEBUG_WRITE), K = 5 / D <= 256 only
  if (nv == 1 && a.debug_write == 1) {
    hipLaunchKernelGGL((k_sgns_atomic<5, 1, 1>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
    return hipGetLastError();
  }
  if (nv == 1 && a.debug_write == 2) {
    hipLaunchKernelGGL((k_sgns_atomic<5, 1, 2>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
    return hipGetLastError();
  }
  if (nv == 1 && a.debug_write == 4) {
    hipLaunchKernelGGL((k_sgns_atomic<5, 1, 4>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
    return hipGetLastError();
  }
  if (nv == 1 && a.debug_write == 5) {
    hipLaunchKernelGGL((k_sgns_atomic<5, 1, 5>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
    return hipGetLastError();
  }
  if (nv == 1 && a.debug_write == 3) {
    hipLaunchKernelGGL((k_sgns_atomic<5, 1, 3>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
    return hipGetLastError();
  }
#endif
  if (a.compute_loss) {
    if (nv == 1)
      hipLaunchKernelGGL((k_sgns_atomic<G2V_K, 1, 0, true>), dim3(grid), dim3(kSgnsThreads), 0, st,
                         a);
    else
      hipLaunchKernelGGL((k_sgns_atomic<G2V_K, 2, 0, true>), dim3(grid), dim3(kSgnsThreads), 0, st,
                         a);
    return hipGetLastError();
  }
  if (nv == 1)
    hipLaunchKernelGGL((k_sgns_atomic<G2V_K, 1>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
  else
    hipLaunchKernelGGL((k_sgns_atomic<G2V_K, 2>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
  return hipGetLastError();
}

int G2V_CAT(sgns_blocks_per_cu_k, G2V_K)(int nv) {
  int nb = 0;
  const hipError_t e =
      nv == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_sgns_atomic<G2V_K, 1>,
                                                             kSgnsThreads, 0)
              : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_sgns_atomic<G2V_K, 2>,
                                                             kSgnsThreads, 0);
  return (e != hipSuccess || nb <= 0) ? 1 : nb;
}

}  // namespace g2v
