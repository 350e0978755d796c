// g2v_sgns.hip -- k_sgns<K,NV,MODE,POL>: the parity/ablation SGNS kernel
// (sequential gensim order, synchronous minibatch, plain-store Hogwild).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "g2v_internal.h"
#include "g2v_device.h"

namespace g2v {

// ---------------------------------------------------------------------------
// k_sgns: one wave per directed example ([ext] fast_sentence_sg_neg)
// ---------------------------------------------------------------------------
// Table traffic goes through buffer resources so every load/store carries an
// explicit cache policy (POL, compile time):
//   kPolPlain   default policy (lines stay in the issuing XCD's L2)
//   kPolWt      stores sc1 (write-through to the coherent side, line dropped
//               from the writer's L2) -- other XCDs see updates within the launch
//   kPolWtRd    kPolWt + sc1 loads
// Rows with vocabulary index < hot_rows (the most frequent genes: indices are
// sorted by descending count) are never stored: their deltas go to the memory
// side as float atomics, one 256-B contiguous wave-instruction per 64 columns,
// so concurrent updates of a hot row are summed, not lost.
template <int K, int NV, int MODE, int POL>
__global__ __launch_bounds__(kSgnsThreads) void k_sgns(SgnsArgs a) {
  __shared__ float s_lut[kExpTableSize];
  __shared__ float s_work[kSgnsThreads / 64][64 * 4 * NV];  // per-wave transpose buffer
  for (int i = threadIdx.x; i < kExpTableSize; i += kSgnsThreads) s_lut[i] = a.exp_table[i];
  __syncthreads();

  constexpr int NT = K + 1;
  constexpr int LA = Pol<POL>::ld, SA = Pol<POL>::st;
  constexpr int NE = NV * 4;  // element-layout columns per lane (l + 64 i)
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  int64_t gw, nw;
  if (MODE == kModeSequential) {
    if (blockIdx.x != 0 || threadIdx.x >= 64) return;
    gw = 0;
    nw = 1;
  } else {
    gw = (int64_t)blockIdx.x * (kSgnsThreads / 64) + wid;
    nw = (int64_t)gridDim.x * (kSgnsThreads / 64);
  }
  const int64_t E = *a.n_examples;
  const int D = a.D;
  const int64_t tbytes = (int64_t)a.V * a.ld * 4;
  const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.rd0, tbytes);
  const __amdgpu_buffer_rsrc_t r1 = make_rsrc(a.rd1, tbytes);
  const __amdgpu_buffer_rsrc_t w0 = make_rsrc(a.wr0, tbytes);
  const __amdgpu_buffer_rsrc_t w1 = make_rsrc(a.wr1, tbytes);
  const int hot = (MODE == kModeSequential || MODE == kModeMinibatch) ? 0 : a.hot_rows;
  const int rowb = (int)a.ld * 4;  // row stride in bytes
  bool on[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) on[v] = (lane + 64 * v) < a.nvec;
  bool eon[NE];
#pragma unroll
  for (int i = 0; i < NE; ++i) eon[i] = (lane + 64 * i) < D;
  // compute_loss: SEQUENTIAL continues gensim's float32 running sum in its
  // order; the parallel modes add each wave's per-chunk float partial in double
  const bool closs = a.compute_loss != 0;
  float lsum = (closs && MODE == kModeSequential) ? *a.loss_f32 : 0.f;

  for (int64_t c = gw; c * kChunk < E; c += nw) {
    const int64_t e_end = (c * kChunk + kChunk < E) ? c * kChunk + kChunk : E;
    for (int64_t e = c * kChunk; e < e_end; ++e) {
      const int32_t* __restrict__ r = a.rec + e * a.rec_stride;
      int32_t tg[NT];
      tg[0] = r[0];
      const int32_t input = r[1];
      const float alpha = __int_as_float(r[2]);
#pragma unroll
      for (int d = 0; d < K; ++d) tg[d + 1] = r[3 + d];

      // gather: syn0[input] (frozen for the example) and the K+1 syn1neg rows
      float4 l1[NV], rw[NT][NV];
      const int in_off = input * rowb + lane * 16;
#pragma unroll
      for (int v = 0; v < NV; ++v)
        l1[v] = on[v] ? bload4<LA>(r0, in_off + 1024 * v) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        const int off = (tg[d] < 0 ? 0 : tg[d]) * rowb + lane * 16;
#pragma unroll
        for (int v = 0; v < NV; ++v)
          rw[d][v] = (on[v] && tg[d] >= 0) ? bload4<LA>(r1, off + 1024 * v)
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      bool any_hot = false;
#pragma unroll
      for (int d = 0; d < NT; ++d) any_hot |= (tg[d] >= 0 && tg[d] < hot);
      // element layout of syn0[input] for coalesced atomics (hot targets only)
      float l1e[NE];
      if (any_hot) {
#pragma unroll
        for (int i = 0; i < NE; ++i)
          l1e[i] = eon[i] ? bload1<LA>(r0, input * rowb + (lane + 64 * i) * 4) : 0.f;
      }

      // K+1 dots, products exact in fp64, summed in fp64 (dsdot semantics)
      double pd[NT], dot[NT];
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        double s = 0.0;
#pragma unroll
        for (int v = 0; v < NV; ++v) s = dot4(l1[v], rw[d][v], s);
        pd[d] = s;
      }
      wave_reduce_multi<NT>(pd, dot, lane);

      float4 work[NV];
#pragma unroll
      for (int v = 0; v < NV; ++v) work[v] = make_float4(0.f, 0.f, 0.f, 0.f);
      bool dirty[NT];
      bool any = false;
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        dirty[d] = false;
        if (tg[d] < 0) continue;
        double dt = dot[d];
        // a repeated target sees its own earlier update (gensim order)
        bool prev_dirty = false;
#pragma unroll
        for (int d2 = 0; d2 < d; ++d2) {
          if (tg[d2] == tg[d]) {
#pragma unroll
            for (int v = 0; v < NV; ++v) rw[d][v] = rw[d2][v];
            prev_dirty = dirty[d2];
          }
        }
        if (prev_dirty) {
          double s = 0.0;
#pragma unroll
          for (int v = 0; v < NV; ++v) s = dot4(l1[v], rw[d][v], s);
          dt = wave_allreduce_d(s);
          dirty[d] = true;
        }
        const float f = (float)dt;
        if (f <= -(float)kMaxExp || f >= (float)kMaxExp) continue;
        const int idx = (int)((f + (float)kMaxExp) * (float)kLutScale);
        const float g = ((d == 0 ? 1.0f : 0.0f) - s_lut[idx]) * alpha;
        if (closs) {
          // [ext] f_dot = (f_dot if d == 0 else -f_dot); loss -= LOG_TABLE[idx(f_dot)]
          const float fl = d == 0 ? f : -f;
          lsum = lsum - a.log_table[(int)((fl + (float)kMaxExp) * (float)kLutScale)];
        }
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          work[v].x = __fmaf_rn(g, rw[d][v].x, work[v].x);
          work[v].y = __fmaf_rn(g, rw[d][v].y, work[v].y);
          work[v].z = __fmaf_rn(g, rw[d][v].z, work[v].z);
          work[v].w = __fmaf_rn(g, rw[d][v].w, work[v].w);
          rw[d][v].x = __fmaf_rn(g, l1[v].x, rw[d][v].x);
          rw[d][v].y = __fmaf_rn(g, l1[v].y, rw[d][v].y);
          rw[d][v].z = __fmaf_rn(g, l1[v].z, rw[d][v].z);
          rw[d][v].w = __fmaf_rn(g, l1[v].w, rw[d][v].w);
        }
        if (tg[d] < hot) {
          float* row = a.wr1 + (int64_t)tg[d] * a.ld + lane;
#pragma unroll
          for (int i = 0; i < NE; ++i)
            if (eon[i]) atomicAdd(row + 64 * i, g * l1e[i]);
        }
        dirty[d] = true;
        any = true;
      }

      // write-back: each touched cold syn1neg row once (its last occurrence)
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        bool later = false;
#pragma unroll
        for (int d2 = d + 1; d2 < NT; ++d2) later |= (tg[d2] == tg[d]);
        if (!dirty[d] || later || tg[d] < hot) continue;
        const int off = tg[d] * rowb + lane * 16;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          if (!on[v]) continue;
          if (MODE == kModeMinibatch) {
            const float4 o = bload4<0>(r1, off + 1024 * v);
            float* p = a.wr1 + (int64_t)tg[d] * a.ld + (lane + 64 * v) * 4;
            atomicAdd(p + 0, rw[d][v].x - o.x);
            atomicAdd(p + 1, rw[d][v].y - o.y);
            atomicAdd(p + 2, rw[d][v].z - o.z);
            atomicAdd(p + 3, rw[d][v].w - o.w);
          } else {
            bstore4<SA>(w1, off + 1024 * v, rw[d][v]);
          }
        }
      }
      if (any) {
        const float lf = a.lockf[input];
        if (input < hot) {
          // transpose work to element layout through LDS, then coalesced atomics
          float* sw = s_work[wid];
#pragma unroll
          for (int v = 0; v < NV; ++v)
            *reinterpret_cast<float4*>(sw + (lane + 64 * v) * 4) = work[v];
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
          float* row = a.wr0 + (int64_t)input * a.ld + lane;
#pragma unroll
          for (int i = 0; i < NE; ++i)
            if (eon[i]) atomicAdd(row + 64 * i, lf * sw[lane + 64 * i]);
          __builtin_amdgcn_wave_barrier();
        } else {
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            if (!on[v]) continue;
            float4 o;
            o.x = __fmaf_rn(lf, work[v].x, l1[v].x);
            o.y = __fmaf_rn(lf, work[v].y, l1[v].y);
            o.z = __fmaf_rn(lf, work[v].z, l1[v].z);
            o.w = __fmaf_rn(lf, work[v].w, l1[v].w);
            if (MODE == kModeMinibatch) {
              float* p = a.wr0 + (int64_t)input * a.ld + (lane + 64 * v) * 4;
              atomicAdd(p + 0, o.x - l1[v].x);
              atomicAdd(p + 1, o.y - l1[v].y);
              atomicAdd(p + 2, o.z - l1[v].z);
              atomicAdd(p + 3, o.w - l1[v].w);
            } else {
              bstore4<SA>(w0, in_off + 1024 * v, o);
            }
          }
        }
      }
    }
    if (closs && MODE != kModeSequential) {
      if (lane == 0 && lsum != 0.f) atomicAdd(a.loss_f64, (double)lsum);
      lsum = 0.f;
    }
  }
  if (closs && MODE == kModeSequential && lane == 0) *a.loss_f32 = lsum;
}


template <int K, int NV, int POL>
static hipError_t launch_sgns_knp(const SgnsArgs& a, int mode, int grid, hipStream_t st) {
  switch (mode) {
    case kModeSequential:
      hipLaunchKernelGGL((k_sgns<K, NV, kModeSequential, POL>), dim3(1), dim3(kSgnsThreads), 0, st,
                         a);
      break;
    case kModeMinibatch:
      hipLaunchKernelGGL((k_sgns<K, NV, kModeMinibatch, POL>), dim3(grid), dim3(kSgnsThreads), 0,
                         st, a);
      break;
    default:
      hipLaunchKernelGGL((k_sgns<K, NV, kModeHogwild, POL>), dim3(grid), dim3(kSgnsThreads), 0, st,
                         a);
  }
  return hipGetLastError();
}


template <int K, int NV>
static hipError_t launch_sgns_kn(const SgnsArgs& a, int mode, int pol, int grid, hipStream_t st) {
  if (mode == kModeHogwild && a.hot_rows >= a.V) {
    return launch_sgns_atomic(a, K, NV, grid, st);
  }
  // sequential / minibatch are parity modes: default policy only
  if (mode == kModeSequential || mode == kModeMinibatch || pol == kPolPlain)
    return launch_sgns_knp<K, NV, kPolPlain>(a, mode, grid, st);
  if (pol == kPolWtRd) return launch_sgns_knp<K, NV, kPolWtRd>(a, mode, grid, st);
  return launch_sgns_knp<K, NV, kPolWt>(a, mode, grid, st);
}


#ifndef G2V_K
#error "g2v_sgns.hip is compiled once per negative count: -DG2V_K=<K>"
#endif
#define G2V_CAT2(a, b) a##b
#define G2V_CAT(a, b) G2V_CAT2(a, b)

hipError_t G2V_CAT(launch_sgns_k, G2V_K)(const SgnsArgs& a, int nv, int mode, int pol, int grid,
                                          hipStream_t st) {
  if (nv == 1) return launch_sgns_kn<G2V_K, 1>(a, mode, pol, grid, st);
  return launch_sgns_kn<G2V_K, 2>(a, mode, pol, grid, st);
}

}  // namespace g2v
