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
// into syn0[input]).  With thousands of examples in flight every row of a
// 24k-gene vocabulary is touched every few microseconds, so plain
// read-modify-write stores lose most updates (measured: iteration-0 loss 4.15
// vs 2.77 sequential); atomics keep all of them (2.76).
//
// Pipelining: a wave takes chunks of kAChunk consecutive
// examples from a work queue and stages each chunk's records and lockf in LDS
// once.  Example e+1's rows are loaded BEFORE example e's atomics are issued
// and after example e-1's have landed (the wave sees its own updates from two
// examples back); e's atomics are a fixed number of buffer atomics, so the
// loop head waits for e+1's rows with vmcnt(#atomics) while e's atomics retire
// behind e+1's compute.  l1 and work are staged through LDS in element order
// so each atomic wave-instruction adds 64 contiguous floats (256 B); the
// row's buffer resource drops the lanes past D.
//
// Build variants: the production library compiles WR 0 (production), 2 (the
// write-free gather roof bench.py measures) and 8 (s_memtime stamps,
// scripts/stamp_segments.py).  The throughput ablations (WR 1, 3, 4, 5, 9 and
// G2V_OPT_DEBUG_WRITE 6 / 7) exist only in the -DG2V_ABLATIONS build
// (gene2vec_amd.build.build(ablations=True) -> gene2vec_amd/libg2v_ablations.so).
// copies of a striped row requested per load batch: all 15 of the top tier's
// extra copies at once for D <= 256 (one memory latency per row instead of
// three; round 5, interleaved A/B: C2 +0.9 %, sample 0 +0.5-1.6 %; round 2's
// kernel had measured no difference), 7 at D > 256 (twice the registers)
#ifndef G2V_STRIPE_BATCH1
#define G2V_STRIPE_BATCH1 15  // (experiment builds override it)
#endif
template <int NV>
constexpr int stripe_batch() { return NV == 1 ? G2V_STRIPE_BATCH1 : 7; }
constexpr int kStripeOob = (int)kStripeMaxBytes;
// examples per work-queue chunk of k_sgns_atomic (<= 64: one lockf per lane
// when the chunk is staged); oracle/c_oracle.py atomic_one_wave(chunk=) follows
#ifndef G2V_CHUNK
#define G2V_CHUNK 32  // (experiment builds override it)
#endif
constexpr int kAChunk = G2V_CHUNK;
static_assert(kAChunk >= 1 && kAChunk <= 64, "one lockf per lane");  // past any stripe buffer (run_sgns clamps rows)

template <int K, int NV>
struct ExRegs {
  int32_t tg[K + 1];
  int32_t input;
  float alpha;
  float4 l1[NV];
  float4 rw[K + 1][NV];
  // a striped hot row's copies, summed in copy order (cs[K + 1]: the syn0
  // row); added to the main row once the main rows have landed (add_copies)
  float4 cs[K + 2][NV];
  bool cp[K + 2];
};

// row t of table tbl (0 = syn0, 1 = syn1neg) as this lane's float4 column(s):
// the main row ...
// Lanes past D read through an out-of-range offset (loff = kLaneOob): the
// buffer range check returns zeros without a memory access, so the loads
// need no exec-masked branch.  Every table is below 2 GiB (g2v_create) and
// the stripe buffer below 1 GiB, so row offset + kLaneOob never wraps.
constexpr uint32_t kLaneOob = 0x80000000u;
template <int NV>
__device__ __forceinline__ void load_main(float4 (&o)[NV], __amdgpu_buffer_rsrc_t rmain, int t,
                                          int rowb, const uint32_t (&loff)[NV]) {
  const uint32_t off = (uint32_t)(t * rowb);
#pragma unroll
  for (int v = 0; v < NV; ++v) o[v] = bload4<0>(rmain, (int)(off + loff[v]));
}

// ... plus its stripe copies when t is a striped hot row (t < stripe_rows).
// The copies are loaded stripe_batch() at a time and summed in copy order, so
// a striped row costs one memory latency per batch, not one per copy; copies
// past stripe_copies read an out-of-range offset (zeros, no memory access).
// t: the row's index within its tier, rows / C: the tier's row count and copies
template <int NV>
__device__ __forceinline__ void add_stripes(float4 (&o)[NV], __amdgpu_buffer_rsrc_t rs, int t,
                                            int tbl, int rows, int C, int rowb,
                                            const uint32_t (&loff)[NV]) {
  constexpr int kStripeBatch = stripe_batch<NV>();
  for (int c0 = 1; c0 < C; c0 += kStripeBatch) {
    float4 q[kStripeBatch][NV];
#pragma unroll
    for (int j = 0; j < kStripeBatch; ++j) {
      const int c = c0 + j;
      const uint32_t base =
          c < C ? (uint32_t)((int)stripe_row(tbl, t, c, rows, C) * rowb) : (uint32_t)kStripeOob;
#pragma unroll
      for (int v = 0; v < NV; ++v) q[j][v] = bload4<0>(rs, (int)(base + loff[v]));
    }
#pragma unroll
    for (int j = 0; j < kStripeBatch; ++j) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        o[v].x += q[j][v].x;
        o[v].y += q[j][v].y;
        o[v].z += q[j][v].z;
        o[v].w += q[j][v].w;
      }
    }
  }
}

// (c mod C) for 0 <= c < C + 32: the stripe copy of a row update without an
// integer division per row
__device__ __forceinline__ int wrap_copy(int c, int C) {
  if (C == 1) return 0;
  while (c >= C) c -= C;
  return c;
}

// destination of an atomic delta for row t of table tbl: the main row or the
// stripe copy (craw mod copies) of its tier (WR 4, ablation build: the same
// rows of a scratch table the kernel never reads).  Byte offsets in 32 bits:
// g2v_create caps a table below 2 GiB (the buffer offset range) and the
// stripe buffers below 1 GiB, so a row's offset is one scalar multiply.
template <int WR = 0>
__device__ __forceinline__ float* upd_row(const SgnsArgs& a, int tbl, int t, int craw, int rowb) {
  if (t >= a.stripe_rows && t < a.stripe2_rows && WR != 4) {
    const int c2 = craw & (a.stripe2_copies - 1);
    if (c2 == 0)
      return reinterpret_cast<float*>(reinterpret_cast<char*>(tbl ? a.wr1 : a.wr0) +
                                      (uint32_t)(t * rowb));
    const int sr =
        (int)stripe_row(tbl, t - a.stripe_rows, c2, a.stripe2_rows - a.stripe_rows,
                        a.stripe2_copies);
    return reinterpret_cast<float*>(reinterpret_cast<char*>(a.stripe2) + (uint32_t)(sr * rowb));
  }
  const int c = wrap_copy(craw, a.stripe_copies);
#ifdef G2V_ABLATIONS
  if (WR == 4) {
    const int64_t nrow = (int64_t)a.V + (int64_t)(a.stripe_copies - 1) * a.stripe_rows;
    const int64_t rr =
        (c == 0 || t >= a.stripe_rows) ? t : a.V + (int64_t)(c - 1) * a.stripe_rows + t;
    return reinterpret_cast<float*>(a.dbg16) + (tbl * nrow + rr) * a.ld;
  }
#endif
  if (c == 0 || t >= a.stripe_rows)
    return reinterpret_cast<float*>(reinterpret_cast<char*>(tbl ? a.wr1 : a.wr0) +
                                    (uint32_t)(t * rowb));
  const int sr = (tbl * a.stripe_rows + t) * (a.stripe_copies - 1) + (c - 1);  // stripe_row()
  return reinterpret_cast<float*>(reinterpret_cast<char*>(a.stripe) + (uint32_t)(sr * rowb));
}

// record e of the chunk staged in LDS (k_sgns_atomic stages each chunk's
// records once): tg / input / alpha as wave-uniform scalars.  The striped hot
// rows' copies are requested FIRST and summed right away (nothing else is in
// flight then: the previous example's atomics have landed), THEN every main
// row is requested and left in flight: the caller issues its atomics behind
// these loads and waits for them only at the next example's first use
// (vmcnt(#atomics)).  Round 3 requested the main rows first and added the
// copies into them here, and that wait on the main rows (the compiler waited
// for all of them before the first copy sum) held every example's atomics
// back by a full load latency (round 4 stamps).
__device__ __forceinline__ uint64_t stamp_time();
template <int K, int NV, bool STAMP = false>
__device__ __forceinline__ void load_example(ExRegs<K, NV>& x, const SgnsArgs& a,
                                             const int32_t* r, __amdgpu_buffer_rsrc_t r0,
                                             __amdgpu_buffer_rsrc_t r1, __amdgpu_buffer_rsrc_t rs,
                                             __amdgpu_buffer_rsrc_t rs2, int rowb,
                                             const uint32_t (&loff)[NV],
                                             uint64_t* t_copies = nullptr) {
  x.tg[0] = __builtin_amdgcn_readfirstlane(r[0]);
  x.input = __builtin_amdgcn_readfirstlane(r[1]);
  x.alpha = __int_as_float(__builtin_amdgcn_readfirstlane(r[2]));
#pragma unroll
  for (int d = 0; d < K; ++d) x.tg[d + 1] = __builtin_amdgcn_readfirstlane(r[3 + d]);
#ifdef G2V_ABLATIONS
  // ablation 6 / 7 (G2V_OPT_DEBUG_WRITE): copies are written but not read (the
  // throughput a drained-copy design would have; values go stale)
  const int R1 = a.skip_copy_reads ? 0 : a.stripe_rows;
  const int R2 = a.skip_copy_reads ? 0 : a.stripe2_rows;
#else
  const int R1 = a.stripe_rows;
  const int R2 = a.stripe2_rows;
#endif
#pragma unroll
  for (int d = 0; d <= K + 1; ++d) {
    const int t = d <= K ? x.tg[d] : x.input;
    const int tbl = d <= K ? 1 : 0;
    x.cp[d] = t >= 0 && t < R2;  // (R2 >= R1)
    if (!x.cp[d]) continue;
#pragma unroll
    for (int v = 0; v < NV; ++v) x.cs[d][v] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t < R1)
      add_stripes<NV>(x.cs[d], rs, t, tbl, R1, a.stripe_copies, rowb, loff);
    else
      add_stripes<NV>(x.cs[d], rs2, t - R1, tbl, R2 - R1, a.stripe2_copies, rowb, loff);
  }
  if (STAMP) *t_copies = stamp_time();  // copies summed (diagnostic build)
  load_main<NV>(x.l1, r0, x.input, rowb, loff);
#pragma unroll
  for (int d = 0; d <= K; ++d) {
    if (x.tg[d] >= 0) {
      load_main<NV>(x.rw[d], r1, x.tg[d], rowb, loff);
    } else {
#pragma unroll
      for (int v = 0; v < NV; ++v) x.rw[d][v] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

// a striped row's value = main + (its copies summed in copy order), once the
// main rows have landed
template <int K, int NV>
__device__ __forceinline__ void add_copies(ExRegs<K, NV>& x) {
#pragma unroll
  for (int d = 0; d <= K + 1; ++d) {
    if (!x.cp[d]) continue;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      float4& o = d <= K ? x.rw[d][v] : x.l1[v];
      o.x += x.cs[d][v].x;
      o.y += x.cs[d][v].y;
      o.z += x.cs[d][v].z;
      o.w += x.cs[d][v].w;
    }
  }
}

// WR: 0 atomics (production), 2 no table writes (the gather roof), 8
// production with s_memtime stamps per loop segment (diagnostic build); in the
// -DG2V_ABLATIONS build also 1 same-shape plain stores, 3 packed-f16 atomics
// into a scratch table (half the atomic bytes, tables never written: a
// throughput probe), 4 the production f32 atomics into that scratch table
// (tables never written), 5 production atomics on syn1neg only, syn0 never
// written (the ceiling of any syn0-side combining), 9 production without each
// row's last atomic instruction (elements 192..255 at D <= 256: a throughput
// probe of the per-wave instruction count; breaks training), 10 production
// with the lost-update probe on every cold-row store (lost_probe)
//
// One row's delta coef * src[0, D) as a FIXED 4 * NV wave-instructions: the
// buffer resource spans the row's D floats, so lanes past D (and every lane of
// a skipped row: live = false gives an empty resource) are dropped by the
// range check and send nothing to memory.  The fixed, branch-free count lets
// the compiler wait for the next example's row loads with vmcnt(#atomics)
// instead of draining this example's atomics (vmcnt(0)) -- atomics retire in
// the background while the wave computes.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(float* row, bool live, int D) {
  // row and live are wave-uniform; say so, or the compiler waterfalls the resource
  const uint64_t pa = reinterpret_cast<uint64_t>(row);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)pa);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(pa >> 32));
  const int nrec = __builtin_amdgcn_readfirstlane(live ? D * 4 : 0);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<float*>(((uint64_t)hi << 32) | lo),
                                           (short)0, nrec, 0x00020000);
}

template <int NV, int WR>
__device__ __forceinline__ void emit_row(float* row, bool live, int D, const float (&src)[4 * NV],
                                         float coef, int lane) {
  const __amdgpu_buffer_rsrc_t r = row_rsrc(row, live, D);
#pragma unroll
  for (int i = 0; i < 4 * NV; ++i) {
#ifdef G2V_ABLATIONS
    if (WR == 9 && i == 4 * NV - 1) continue;  // ablation: no tail instruction
#endif
    const int off = (64 * i + lane) * 4;
    const float v = coef * src[i];
    if (WR == 0 || WR == 4 || WR == 5 || WR == 8 || WR == 9 || WR == 10)
      __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v, r, off, 0, 0);
    else if (WR == 1)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 0);
  }
}

// G2V_OPT_TAIL_STORE: a cold row (syn0 index >= a.tail_row0,
// syn1neg index >= a.tail_row1, never a striped row; syn1neg rows only in a
// repeat-free example) is written with plain stores of its new value instead
// of float atomics of the delta, write-through (sc1: the line leaves the
// writer's L2, so a later read on that XCD fetches the memory side's copy).
// gensim's own Hogwild read-modify-write, with the lost updates that implies
// when another wave wrote the row between this wave's read and its store --
// which is why only rows that other in-flight waves rarely touch take it
// (run_sgns's collision budget).
//
// The row leaves as 16-B lanes: its nvec float4 columns (element 4 c .. 4 c + 3
// in lane c mod 64 of vector c / 64), NV b128 instructions, plus 3 NV stores
// through an empty resource that the range check drops whole (nothing reaches
// memory), so both sides of the store-or-atomics if / else count 4 NV
// vector-memory instructions for the loop head's vmcnt.  (Round 5 A/B against
// 4 NV b32 stores: C4 +1.3 %, C2 equal; the b32 form was removed.)  The columns
// past D inside the last float4 are the tables' zero padding, which every
// float4 kernel (loads, merges) already carries.
template <int NV>
__device__ __forceinline__ void store_row4(float* row, bool live, int nvec,
                                           const float4 (&val)[NV], int lane) {
  const __amdgpu_buffer_rsrc_t r = row_rsrc(row, live, 4 * nvec);
  const __amdgpu_buffer_rsrc_t rz = row_rsrc(row, false, 0);
#pragma unroll
  for (int v = 0; v < NV; ++v) bstore4<Pol<kPolWt>::st>(r, (lane + 64 * v) * 16, val[v]);
#pragma unroll
  for (int i = 0; i < 3 * NV; ++i)  // distinct offsets, or they merge as dead stores
    __builtin_amdgcn_raw_buffer_store_b32(0u, rz, (64 * i + lane) * 4, 0, 0);
}

#ifdef G2V_ABLATIONS
// WR 10 (ablation build): before a cold row's store, re-read its first 64
// floats write-through-fresh (sc1: past this CU's L1) and compare them with
// the values this wave read for its update (old = element `lane`); a
// difference means another wave wrote the row inside this wave's read-to-
// store window, and the store about to land overwrites that update -- one
// lost update.  stamps[14] += stores probed, stamps[15] += rows changed.
__device__ __forceinline__ void lost_probe(float* row, float old, unsigned long long* stamps,
                                           int lane) {
  const __amdgpu_buffer_rsrc_t r = row_rsrc(row, true, 64);
  const float now = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, lane * 4, 0, 16));
  const bool changed = __builtin_amdgcn_ballot_w64(now != old) != 0;
  if (lane == 0) {
    atomicAdd(stamps + 14, 1ull);
    if (changed) atomicAdd(stamps + 15, 1ull);
  }
}
#endif

// LOSS ([ext] compute_loss): each wave keeps a float32 partial of the
// -log(sigmoid(+-f)) LOG_TABLE terms over its chunk and adds it to a double
// accumulator once per chunk; LOSS = false compiles the tally out.
// Chunks of kAChunk consecutive examples are handed out by a work queue (one
// counter, lane 0's returning atomic): every wave works near the front of
// the record stream whatever its speed.  With a static grid-stride split,
// waves that share a CU (grid not a multiple of the CU count) fall behind
// and apply early, high-alpha examples to a model the others have already
// moved on: C2 vocabulary at 266 workgroups drifted +0.42 % from the
// sequential objective, 256 and 300 stayed within 0.1 %.
// a value every lane holds alike (a wave_allreduce_d total) as a scalar: the
// compiler cannot prove the butterfly's result uniform, and a branch on it
// would turn every later row choice into exec-masked VALU work (round 2: ~55
// instructions per row update, most of them address arithmetic)
__device__ __forceinline__ float uniform_f(float x) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}
__device__ __forceinline__ bool uniform_b(bool x) {
  return __builtin_amdgcn_readfirstlane((int)x) != 0;
}

// In-kernel stamps (WR 8 only; cdna_hip_programming.md 7 "In-kernel stamps"):
// one asm statement per stamp, the lgkmcnt(0) inside it, fenced from the
// scheduler on both sides.  Read the segment SHARES of such a build, never its
// run time (the fences forbid overlaps the production kernel has).
__device__ __forceinline__ uint64_t stamp_time() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
__device__ __forceinline__ uint64_t stamp_realtime() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
// s_waitcnt immediate (gfx9 layout) for vmcnt(n), lgkmcnt / expcnt not waited
constexpr int waitcnt_vm(int n) { return 0x0F70 | (n & 0xF) | (((n >> 4) & 3) << 14); }

__device__ __forceinline__ int64_t next_chunk(unsigned int* q, int lane) {
  unsigned int v = 0;
  if (lane == 0) v = atomicAdd(q, 1u);
  return (int64_t)__builtin_amdgcn_readfirstlane(v);
}

// tail stores stage the new values of up to kTailSlots cold syn1neg rows per
// example in LDS (later cold rows of the example take atomics): 6 KB per wave
// at negative 5 / D <= 256, 16 KB at D > 256 with 8 or more targets
constexpr int kTailSlots = 8;

template <int K, int NV, int WR = 0, bool LOSS = false>
__global__ __launch_bounds__(kSgnsThreads) void k_sgns_atomic(SgnsArgs a) {
  constexpr int NT = K + 1;
  constexpr int W = kSgnsThreads / 64;
  constexpr int RS = (3 + K + 3) / 4 * 4;  // record stride (g2v_create: 16-B records)
  // tail stores compiled in (WR 8: the stamped production build; WR 10,
  // ablation build: with the lost-update probe)
  constexpr bool TS = WR == 0 || WR == 8 || WR == 10;
  constexpr int kSlots = NT < kTailSlots ? NT : kTailSlots;
  __shared__ float s_lut[kExpTableSize];
  __shared__ float s_log[LOSS ? kExpTableSize : 1];
  __shared__ float s_l1[W][256 * NV];
  __shared__ float s_wk[W][256 * NV];
  __shared__ float s_tl[W][TS ? kSlots * 256 * NV : 1];  // tail rows' new values (TS)
  __shared__ float s_to[W][WR == 10 ? kSlots * 64 : 1];  // WR 10: their old first 64 floats
  __shared__ int32_t s_rec[W][kAChunk * RS];  // the wave's chunk of records
  __shared__ float s_lf[W][kAChunk];          // lockf[input] per record of the chunk
  for (int i = threadIdx.x; i < kExpTableSize; i += kSgnsThreads) {
    s_lut[i] = a.exp_table[i];
    if (LOSS) s_log[i] = a.log_table[i];
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // G2V_OPT_ACTIVE_WAVES (parity checks): with 1 wave on a 1-workgroup grid the
  // chunks train in record order and the update order is a fixed function of
  // the records, restated in oracle/sgns_oracle.c (oracle_atomic_one_wave)
  if (wid >= a.active_waves) return;
  {
    // stability cap: a hot syn0 row's in-flight updates scale
    // with waves x p_tok x (K+1) x alpha x |syn1neg|^2; from the norm measured
    // just before this launch, only the first `cap` waves (spread wave-major
    // over the workgroups, so as many CUs as possible keep one) train
    int cap = (int)gridDim.x * a.active_waves;
    if (a.norm_bits != nullptr) {
      const float per_wave = a.cap_coef * __uint_as_float(*a.norm_bits);
      if (per_wave > 0.f) {
        const float w = a.cap_budget / per_wave;
        if (w < (float)cap) cap = w < 1.f ? 1 : (int)w;
      }
    }
    if (a.waves_out != nullptr && blockIdx.x == 0 && wid == 0 && lane == 0) *a.waves_out = cap;
    if (wid * (int)gridDim.x + (int)blockIdx.x >= cap) return;
  }
  const int64_t E = *a.n_examples;
  const int D = a.D;
  const int64_t tbytes = (int64_t)a.V * a.ld * 4;
  const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.rd0, tbytes);
  const __amdgpu_buffer_rsrc_t r1 = make_rsrc(a.rd1, tbytes);
  const __amdgpu_buffer_rsrc_t rs =
      make_rsrc(a.stripe, 2 * (int64_t)(a.stripe_copies - 1) * a.stripe_rows * a.ld * 4);
  const __amdgpu_buffer_rsrc_t rs2 =
      make_rsrc(a.stripe2, a.stripe2_rows > a.stripe_rows
                               ? 2 * (int64_t)(a.stripe2_copies - 1) *
                                     (a.stripe2_rows - a.stripe_rows) * a.ld * 4
                               : 0);
  const int rowb = (int)a.ld * 4;
  // first cold row taking plain stores (V or more: none; run_sgns keeps it
  // past both stripe tiers)
  const int tail0 = TS ? a.tail_row0 : 0x7fffffff;
  const int tail1 = TS ? a.tail_row1 : 0x7fffffff;
  float* s1 = s_l1[wid];
  float* sw = s_wk[wid];
  float* stl = s_tl[wid];
  int32_t* sr = s_rec[wid];
  float* slf = s_lf[wid];
  uint32_t loff[NV];  // this lane's byte offset in a row, out of range past D
#pragma unroll
  for (int v = 0; v < NV; ++v)
    loff[v] = (lane + 64 * v) < a.nvec ? (uint32_t)(lane * 16 + 1024 * v) : kLaneOob;

  // WR 8: cycle sums per segment (see g2v_debug_stamps), wave-uniform scalars
  constexpr int kAtomicsPerExample = 4 * NV * (NT + 1);  // emit_row's fixed count
  uint64_t acc[5] = {0, 0, 0, 0, 0};
  uint64_t sub[4] = {0, 0, 0, 0};  // dots+reduce, LUT/gradients, first 4 rows' atomics, copies
  uint64_t n_ex = 0, tl0 = 0, rl0 = 0;
  if (WR == 8) {
    rl0 = stamp_realtime();
    tl0 = stamp_time();
  }
  for (int64_t c = next_chunk(a.queue, lane); c * kAChunk < E; c = next_chunk(a.queue, lane)) {
    const int64_t e_beg = c * kAChunk;
    const int64_t e_end = (e_beg + kAChunk < E) ? e_beg + kAChunk : E;
    // stage the chunk's records and their lockf once: per example, only row
    // loads and atomics are vector-memory operations
    {
      const int nint = (int)(e_end - e_beg) * RS;
      const int32_t* rb = a.rec + e_beg * RS;
      for (int i = lane; i < nint; i += 64) sr[i] = rb[i];
      __builtin_amdgcn_wave_barrier();
      if (lane < e_end - e_beg) slf[lane] = a.lockf[sr[lane * RS + 1]];
      __builtin_amdgcn_wave_barrier();
    }
    // stripe copy of example e's first row update: (e + d) mod copies, advanced
    // per example (no division in the loop)
    int cbase = (int)(e_beg % (int64_t)a.stripe_copies);
    float lsum = 0.f;
    ExRegs<K, NV> x;
    load_example<K, NV>(x, a, sr, r0, r1, rs, rs2, rowb, loff);
    // drain here, so the loop head only waits on the back edge's count
    // (vmcnt(#atomics of the previous example)); without it the two incoming
    // paths merge to vmcnt(0), which also waits for the previous atomics
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    for (int64_t e = e_beg; e < e_end; ++e) {
      const int q = (int)(e - e_beg);
      if (!a.overlap) __builtin_amdgcn_s_waitcnt(0x0F70);  // e-1's atomics land first
      uint64_t ts = 0;
      if (WR == 8) {
        // the wait production makes at its first use of e's rows, made explicit
        const uint64_t t0 = stamp_time();
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(kAtomicsPerExample));
        ts = stamp_time();
        acc[0] += ts - t0;
        ++n_ex;
      }
      // ---- compute example e ------------------------------------------------
      add_copies<K, NV>(x);
      double pd[NT], dot[NT];
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        double s = 0.0;
#pragma unroll
        for (int v = 0; v < NV; ++v) s = dot4(x.l1[v], x.rw[d][v], s);
        pd[d] = s;
      }
      wave_reduce_multi<NT>(pd, dot, lane);
      uint64_t tsub = 0;
      if (WR == 8) {
        tsub = stamp_time();
        sub[0] += tsub - ts;
      }
      float4 work[NV];
#pragma unroll
      for (int v = 0; v < NV; ++v) work[v] = make_float4(0.f, 0.f, 0.f, 0.f);
      // sigmoid (and LOG_TABLE) lookups of all K+1 dots issued together, not
      // one dependent LDS round trip per row; a duplicate of an updated row
      // recomputes its dot and looks up again below
      float fv[NT], lv[NT], lg[NT];
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        fv[d] = uniform_f((float)dot[d]);
        const bool in = fv[d] > -(float)kMaxExp && fv[d] < (float)kMaxExp;
        lv[d] = s_lut[in ? (int)((fv[d] + (float)kMaxExp) * (float)kLutScale) : 0];
        if (LOSS) {
          const float fl = d == 0 ? fv[d] : -fv[d];
          lg[d] = s_log[in ? (int)((fl + (float)kMaxExp) * (float)kLutScale) : 0];
        }
      }
      float g[NT];
      bool live[NT];  // wave-uniform: row d takes an update
      bool dirty[NT];
      bool any = false;
      // a target repeated within the example (a negative equal to an earlier
      // target) takes the general path below, which applies the repeats in
      // order; without repeats (most examples: a few % have one at sample 0)
      // the rows are independent and their updated values are never read
      // again (the atomics send g * l1), so only work accumulates -- the
      // per-row repeat logic was most of the 2,090 cycles this section took
      // per example (round 4 stamps)
      bool rep = false;
#pragma unroll
      for (int d = 1; d < NT; ++d)
#pragma unroll
        for (int d2 = 0; d2 < d; ++d2) rep |= x.tg[d2] == x.tg[d];  // (-1 pads: general path)
      // per target: its LDS staging slot when the row is stored (a cold row of
      // a repeat-free example, while slots last), -1 = float atomics
      int slot[NT];
#pragma unroll
      for (int d = 0; d < NT; ++d) slot[d] = -1;
      int nslot = 0;
      if (!rep) {
#pragma unroll
        for (int d = 0; d < NT; ++d) {
          g[d] = 0.f;
          live[d] = false;
          const float f = fv[d];
          if (x.tg[d] < 0 || f <= -(float)kMaxExp || f >= (float)kMaxExp) continue;
          const float gg = ((d == 0 ? 1.0f : 0.0f) - lv[d]) * x.alpha;
          if (LOSS) lsum = lsum - lg[d];
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            work[v].x = __fmaf_rn(gg, x.rw[d][v].x, work[v].x);
            work[v].y = __fmaf_rn(gg, x.rw[d][v].y, work[v].y);
            work[v].z = __fmaf_rn(gg, x.rw[d][v].z, work[v].z);
            work[v].w = __fmaf_rn(gg, x.rw[d][v].w, work[v].w);
          }
          if (TS && x.tg[d] >= tail1 && nslot < kSlots) {
            // the cold row's new value, staged in element order for store_row4
            if (WR == 10 && lane < 16)
              *reinterpret_cast<float4*>(s_to[wid] + nslot * 64 + lane * 4) = x.rw[d][0];
#pragma unroll
            for (int v = 0; v < NV; ++v) {
              float4 nw;
              nw.x = __fmaf_rn(gg, x.l1[v].x, x.rw[d][v].x);
              nw.y = __fmaf_rn(gg, x.l1[v].y, x.rw[d][v].y);
              nw.z = __fmaf_rn(gg, x.l1[v].z, x.rw[d][v].z);
              nw.w = __fmaf_rn(gg, x.l1[v].w, x.rw[d][v].w);
              *reinterpret_cast<float4*>(stl + nslot * 256 * NV + (lane + 64 * v) * 4) = nw;
            }
            slot[d] = nslot++;
          }
          g[d] = gg;
          live[d] = true;
          any = true;
        }
      } else {
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        g[d] = 0.f;
        live[d] = false;
        dirty[d] = false;
        if (x.tg[d] < 0) continue;
        bool prev_dirty = false;
#pragma unroll
        for (int d2 = 0; d2 < d; ++d2) {
          if (x.tg[d2] == x.tg[d]) {
#pragma unroll
            for (int v = 0; v < NV; ++v) x.rw[d][v] = x.rw[d2][v];
            prev_dirty = dirty[d2];
          }
        }
        float f = fv[d], lut = lv[d], lgv = LOSS ? lg[d] : 0.f;
        if (prev_dirty) {
          double s = 0.0;
#pragma unroll
          for (int v = 0; v < NV; ++v) s = dot4(x.l1[v], x.rw[d][v], s);
          f = uniform_f((float)wave_allreduce_d(s));
          dirty[d] = true;
          if (f > -(float)kMaxExp && f < (float)kMaxExp) {
            lut = s_lut[(int)((f + (float)kMaxExp) * (float)kLutScale)];
            if (LOSS) {
              const float fl = d == 0 ? f : -f;
              lgv = s_log[(int)((fl + (float)kMaxExp) * (float)kLutScale)];
            }
          }
        }
        if (f <= -(float)kMaxExp || f >= (float)kMaxExp) continue;
        const float gg = ((d == 0 ? 1.0f : 0.0f) - lut) * x.alpha;
        if (LOSS) lsum = lsum - lgv;
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
        live[d] = true;
        dirty[d] = true;
        any = true;
      }
      }
      if (WR == 8) {
        const uint64_t t = stamp_time();
        sub[1] += t - tsub;
      }
      // stage l1 / work in element order
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        *reinterpret_cast<float4*>(s1 + (lane + 64 * v) * 4) = x.l1[v];
        *reinterpret_cast<float4*>(sw + (lane + 64 * v) * 4) = work[v];
      }
      __builtin_amdgcn_wave_barrier();
      // this lane's elements 64 i + lane of l1 and work, read back once for all rows
      float v1[4 * NV], vw[4 * NV];
#pragma unroll
      for (int i = 0; i < 4 * NV; ++i) {
        v1[i] = s1[64 * i + lane];
        vw[i] = sw[64 * i + lane];
      }
      int32_t tg[NT];
#pragma unroll
      for (int d = 0; d < NT; ++d) tg[d] = x.tg[d];
      const int32_t input = x.input;
      const float lf = slf[q];
      if (WR == 8) {
        const uint64_t t = stamp_time();
        acc[1] += t - ts;
        ts = t;
      }

      // ---- prefetch example e+1 (its loads overtake e's atomics) -------------
      // e-1's atomics retired behind e's compute; they must have landed before
      // e+1 reads rows (a wave sees its own updates two examples back, as
      // before this pipelining: the Hogwild staleness stays what the grid
      // budget was measured with)
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      if (WR == 8) {
        const uint64_t t = stamp_time();
        acc[2] += t - ts;
        ts = t;
      }
      uint64_t tmain = ts;
      if (e + 1 < e_end)
        load_example<K, NV, WR == 8>(x, a, sr + (q + 1) * RS, r0, r1, rs, rs2, rowb, loff,
                                     &tmain);
      if (WR == 8) sub[3] += tmain - ts;
      if (WR == 8) {
        const uint64_t t = stamp_time();
        acc[3] += t - ts;
        ts = t;
      }

      // ---- atomics of example e -----------------------------------------------
#ifdef G2V_ABLATIONS
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
        cbase = cbase + 1 == a.stripe_copies ? 0 : cbase + 1;
        continue;
      }
#endif
      // syn1neg[tg[d]] += g[d] * l1 (d = 0..K), then syn0[input] += lockf * work;
      // a cold row (G2V_OPT_TAIL_STORE) takes its stores INSTEAD: a uniform
      // if / else with 4 NV vector-memory instructions on each side (store_row4
      // pads its NV 16-B stores with dropped ones),
      // so the loop head waits for the next example's loads with
      // vmcnt(#row instructions).  That needs the build's
      // -structurizecfg-skip-uniform-regions (gene2vec_amd/build.py): the
      // default structurizer lowers the if / else to two triangles, and the
      // path through neither made the loop head wait with vmcnt(0) (every
      // atomic of the previous example drained before the next compute);
      // tests/test_kernel_isa.py checks the wait in the assembly
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        float* row = upd_row<WR>(a, 1, live[d] ? tg[d] : 0, cbase + d, rowb);
        const bool st = uniform_b(TS && slot[d] >= 0);
        if (st) {
#ifdef G2V_ABLATIONS
          if (WR == 10 && live[d]) lost_probe(row, s_to[wid][slot[d] * 64 + lane], a.stamps, lane);
#endif
          float4 val[NV];
#pragma unroll
          for (int v = 0; v < NV; ++v)
            val[v] = *reinterpret_cast<const float4*>(stl + slot[d] * 256 * NV + (lane + 64 * v) * 4);
          store_row4<NV>(row, live[d], a.nvec, val, lane);
        } else {
          emit_row<NV, WR>(row, live[d], D, v1, g[d], lane);
        }
        if (WR == 8 && d == 3) sub[2] += stamp_time() - ts;  // 16 atomics issued
      }
      {
        float* row = upd_row<WR>(a, 0, input, cbase + NT, rowb);
        const bool st = uniform_b(TS && input >= tail0);
        if (st) {
#ifdef G2V_ABLATIONS
          if (WR == 10 && any) lost_probe(row, v1[0], a.stamps, lane);
#endif
          float4 val[NV];
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            const float4 l = *reinterpret_cast<const float4*>(s1 + (lane + 64 * v) * 4);
            const float4 w = *reinterpret_cast<const float4*>(sw + (lane + 64 * v) * 4);
            val[v] = make_float4(__fmaf_rn(lf, w.x, l.x), __fmaf_rn(lf, w.y, l.y),
                                 __fmaf_rn(lf, w.z, l.z), __fmaf_rn(lf, w.w, l.w));
          }
          store_row4<NV>(row, any, a.nvec, val, lane);
        } else {
          emit_row<NV, WR>(row, any && WR != 5, D, vw, lf, lane);
        }
      }
      __builtin_amdgcn_wave_barrier();
      if (WR == 8) acc[4] += stamp_time() - ts;
      cbase = cbase + 1 == a.stripe_copies ? 0 : cbase + 1;
    }
    if (LOSS && lane == 0 && lsum != 0.f) atomicAdd(a.loss_f64, (double)lsum);
  }
  if (WR == 8) {
    const uint64_t tl = stamp_time() - tl0;
    const uint64_t rl = stamp_realtime() - rl0;
    if (lane == 0) {
      unsigned long long* o = a.stamps;
      for (int i = 0; i < 5; ++i) atomicAdd(o + i, (unsigned long long)acc[i]);
      atomicAdd(o + 5, (unsigned long long)tl);
      atomicAdd(o + 6, (unsigned long long)n_ex);
      atomicAdd(o + 7, (unsigned long long)tl);
      atomicAdd(o + 8, (unsigned long long)rl);
      atomicAdd(o + 9, 1ull);
      for (int i = 0; i < 4; ++i) atomicAdd(o + 10 + i, (unsigned long long)sub[i]);
    }
  }
}


#ifndef G2V_K
#error "g2v_sgns_atomic.hip is compiled once per negative count: -DG2V_K=<K>"
#endif
#define G2V_CAT2(a, b) a##b
#define G2V_CAT(a, b) G2V_CAT2(a, b)

// the instance a launch runs (run_sgns has already refused a debug mode this
// shape does not compile: g2v_set_option, G2V_OPT_DEBUG_WRITE)
hipError_t G2V_CAT(launch_sgns_atomic_k, G2V_K)(const SgnsArgs& a, int nv, int grid,
                                                 hipStream_t st) {
#if G2V_K == 5
  // the gather roof and the stamped diagnostic build, K = 5 / D <= 256 only
  if (nv == 1 && a.debug_write == 2) {
    hipLaunchKernelGGL((k_sgns_atomic<5, 1, 2>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
    return hipGetLastError();
  }
  if (nv == 1 && a.debug_write == 8) {
    hipLaunchKernelGGL((k_sgns_atomic<5, 1, 8>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
    return hipGetLastError();
  }
#ifdef G2V_ABLATIONS
  if (nv == 1 && a.debug_write == 1) {
    hipLaunchKernelGGL((k_sgns_atomic<5, 1, 1>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
    return hipGetLastError();
  }
  if (nv == 1 && a.debug_write == 3) {
    hipLaunchKernelGGL((k_sgns_atomic<5, 1, 3>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
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
  if (nv == 1 && a.debug_write == 9) {
    hipLaunchKernelGGL((k_sgns_atomic<5, 1, 9>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
    return hipGetLastError();
  }
  if (nv == 1 && a.debug_write == 10) {
    hipLaunchKernelGGL((k_sgns_atomic<5, 1, 10>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
    return hipGetLastError();
  }
#endif
#endif
#if G2V_K == 15 && defined(G2V_ABLATIONS)
  if (nv == 2 && a.debug_write == 10) {  // the lost-update probe at the C4 shape
    hipLaunchKernelGGL((k_sgns_atomic<15, 2, 10>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
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
