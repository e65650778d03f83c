// Fused SDF / moment "tower" kernels on the compacted panel (one row = one valid (t, i)).
//
// Replaces the reference hot path `SDFNetwork.forward` + `MomentNetwork.forward` and their
// autograd (`/root/reference/src/model.py:132-161,221-281,513-521`, profile in SURVEY §2.3
// K1/K2/K4/K12): macro tiling + cat + Linear/ReLU/Dropout x L + output projection + mask
// become ONE kernel per direction; activations stay in registers; dropout masks come from a
// counter hash (recomputed in backward, never stored).
//
// Widths are padded at pack time (zero weights/biases are exact no-ops through ReLU):
//   SDF tower: every hidden layer is 64 units (4 blocks of 16);
//   moment tower: every layer is WM = 16*WMB units (WMB in {1,2,4}, template).
// Layer 0 reads KP = 32*KS1 panel columns (KS1 in {2,4}, template).
//
// ---- Data orientation -----------------------------------------------------------------
// A wave owns a 32-row tile = 2 row blocks (b = 0, 1) of 16 rows. Everything is computed in
// the "T" orientation: an activation block is a 16(units) x 16(rows) MFMA C tile,
//      lane l holds  act[unit = 16u + 4*(l>>4) + r][row = l & 15],  r = 0..3.
// Layer 0:   Z0^T = W0 . X^T           A = W0 frag (natural k), B = X frag
//            (lane l: X[row l&15][k = 32s + 8q + j] -- a plain 16-byte load of the row).
// Layer j:   Zj^T = Wj . A(j-1)^T      B = two C blocks packed (pack8): the k order inside a
//            step is permuted, k(q, j) = j < 4 ? 4q + j : 16 + 4q + (j-4); the packed weight
//            fragment uses the same permutation, so no lane movement is needed.
// Backward chain dA(j-1)^T = Wj^T . dZj^T: the identical trick with the transposed blob.
// Weight gradients dW = sum_rows dZ . A^T need rows on the k axis: the A and B operand maps
// are mirror images, so an MFMA of a packed T fragment (as A) against a 0/1 selector (as B)
// *transposes* a 16x16 block exactly (bf16 x 1.0, one non-zero term per output):
//      N layout: lane l holds act[unit = 16c + (l&15)][row = 4*(l>>4) + r].
// Packing the two row blocks' N tiles gives operands whose k axis is the tile's 32 rows
// (k(q, j) = row 4q + (j&3) of block j>>2), so dW tiles accumulate in registers across the
// whole persistent loop. Bias sums use the same rows-as-k operands against a one-hot
// column selector: every layer's bias gradient shares 4 accumulator tiles.
#include <algorithm>
#include "common.h"
#include "layout.h"
#include "mlp.h"
#include "lstm_gls.h"
#include "tower_dev.h"

// Waves per SIMD the forward tower kernel is compiled for (its VGPR budget = 512 / this).
#ifndef DLAP_FWD_WPS
#define DLAP_FWD_WPS 2
#endif

// Waves per SIMD of the one-tile-per-slice SDF backward (TPS = 1): 2 halves its register budget
// and lets two waves hide each other's MFMA / LDS latency (600x3000x46: 0.1983 vs 0.2041 ms
// per epoch for the two-tiles-per-slice kernel at one wave, profiles/r4_bwd_shape.log).
#ifndef DLAP_BWD1_WPS
#define DLAP_BWD1_WPS 2
#endif

// In-kernel timestamps (wall clock, 100 MHz) of k_mlp_fwd's first / last workgroup, wave 0:
// [0] start, [1] weights staged, [2] first tile done, [3] loop done; [4..7] same, last block.
// [8..12]: fused LSTM + tower forward, workgroup 0: start, recurrence start / end, LSTM body
// done, publisher done (k_mlp_fwd_rnn).
__device__ long long g_mlp_ts[24];   // [16..]: the last evaluation recurrence (fused forward)
#define MLP_TS(slot) do { \
    if ((threadIdx.x & 255) == 0 && (bx == 0 || bx == gxw - 1) && J.gbits) \
      g_mlp_ts[(bx == 0 ? 0 : 4) + (slot)] = wall_clock64(); } while (0)
// SDF tower forward on one tile: the raw (pre-normalisation) weight of each row block.
// kw[j]: keep word of hidden layer j (ignored unless DROP). layer0_fn(a) fills the layer-0
// pre-activations including the bias (fused: MFMA over the X tile; wide: from z).
// Output layer on the matrix cores: the 2 s_wo fragments hold the output row as row 0 of an
// A operand, so C[0][row] = wo . act + bo lands on the lanes of lane group 0.
template <class P, bool DROP, typename L0>
DLAP_DEV void sdf_forward_tile(const typename P::Frag* lds, const float* aux, const MlpDims& D,
                               const uint32_t (&kw)[4], L0&& layer0_fn, float (&w)[2]) {
  f32x4 a[2][4];
  typename P::Frag pf[2][2];
  layer0_fn(a);
  act_tile<P, 4, DROP>(a, kw[0], pf);
  // fully unrolled to the engine's 4-layer limit so kw[j] is a register, not scratch
#pragma unroll
  for (int j = 1; j < 4; ++j) {
    if (j >= D.nl_sdf) break;
    layer_chain<P, 4, 2>(lds, D.s_fwd + (j - 1) * 8, pf, a, aux + D.a_sb + 64 * j);
    act_tile<P, 4, DROP>(a, kw[j], pf);
  }
  const int q = lane_id() >> 4;
  const float bo = aux[D.a_bo];
  f32x4 c0 = f32x4{q == 0 ? bo : 0.f, 0.f, 0.f, 0.f}, c1 = c0;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const typename P::Frag wf = ldsf(lds, D.s_wo + s);
    c0 = P::mma(wf, pf[0][s], c0);
    c1 = P::mma(wf, pf[1][s], c1);
  }
  w[0] = c0[0];
  w[1] = c1[0];
}

// Moment tower forward on one tile: writes the K tanh outputs of every valid row. layer0_fn
// fills the layer-0 pre-activations including the per-period bias.
template <class P, int WMB, typename L0>
DLAP_DEV void mom_forward_tile(const typename P::Frag* lds, const float* aux, const MlpDims& D,
                               const MlpJob& J, const DropCtx& dc, const RowInfo& ri, L0&& layer0_fn) {
  constexpr int KSM = (WMB + 1) / 2;
  f32x4 a[2][WMB];
  typename P::Frag pf[2][KSM];
  const int q = lane_id() >> 4;
  layer0_fn(a);
  for (int j = 0; j + 1 < D.nl_mom; ++j) {
    const uint32_t kw = dc.on ? hash_keep<WMB>(dc, 16 + j, ri) : 0xFFFFFFFFu;
    act_tile_rt<P, WMB>(a, dc.on, kw, pf);
    layer_chain<P, WMB, KSM>(lds, D.m_fwd + j * WMB * KSM, pf, a, aux + D.a_mb + 64 * (j + 1));
  }
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    if (ri.dense[b] < 0) continue;
    const auto dst = gp(J.h_out) + (size_t)ri.dense[b] * D.K;
#pragma unroll
    for (int u = 0; u < WMB; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = 16 * u + 4 * q + r;
        if (k < D.K) dst[k] = tanhf(a[b][u][r]);
      }
  }
}

// ============================== forward ==================================================
// Keep words of the SDF hidden layers for one tile: pre-generated (pre), hashed, or all kept.
DLAP_DEV void sdf_keep_words(bool pre, const uint32_t (&kw_pre)[4], const DropCtx& dc, const RowInfo& ri,
                             int nl, uint32_t (&kw)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (pre) kw[j] = kw_pre[j];
    else if (dc.on && j < nl) kw[j] = hash_keep<4>(dc, j, ri);
    else kw[j] = 0xFFFFFFFFu;
  }
}

// Bounded spin on the fused forward's progress counter (k_mlp_fwd_rnn): wave-uniform, s_sleep
// between polls. The engine launches the fused forward only when its whole grid is co-resident
// (occupancy query, engine.cpp fused_fits), so the wait always ends; it is bounded anyway
// (~0.1 s, MlpJob::prog_limit): a wave that gives up counts it in *err and returns -1, and the
// caller then stops WITHOUT writing anything -- the launch is invalid, k_adam skips the update
// and k_epoch_end records a NaN epoch for that model (the device-side poison), and the host
// raises at its next synchronisation (runner.py). Nothing is ever computed on unpublished data.
DLAP_DEV int prog_wait(const int* prog, int* err, int need, int seen, bool fence, unsigned limit) {
  if (need <= seen) return seen;
  int v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  unsigned spins = 0;
  while (v < need) {
    if (spins++ >= limit) {
      if ((threadIdx.x & 63) == 0) atomicAdd(err, 1);
      return -1;
    }
    __builtin_amdgcn_s_sleep(2);
    v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
  // Compiler-only barrier: the relaxed loads of the published outputs (finish_tile FRESH) must
  // not be hoisted above the poll that decided the exit (different addresses, so the language
  // model alone would allow it). The hardware order follows from the exit branch waiting for
  // the poll's value. Costs no instruction.
  asm volatile("" ::: "memory");
  // the outputs published before the counter are visible to this wave's loads from here on
  // (prog mode 0; mode 1 reads them with cache-bypassing loads instead of invalidating)
  if (fence) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return v;
}

// Tower forward over the tiles of workgroup `bx` of `gxw` (k_mlp_fwd: the whole grid.x; the
// fused k_mlp_fwd_rnn: grid.x - 1, its workgroup 0 runs the LSTM). WAIT: the per-period inputs
// are produced concurrently by that LSTM -- before a tile is finished, the wave waits until the
// periods of its rows are published (J.prog) and reads them from global memory.
// SO: the SDF tower only, with its dropout masks pre-generated (or no dropout) -- the phase-1/3
// training forward and the evaluation forward of the epoch graphs. The moment tower and the
// in-kernel mask hash are compiled out, so the tile loop carries neither their branches nor
// their registers (the host picks SO only when every job qualifies: launch_mlp_fwd*).
template <class P, int KS1, int WMB, bool ZIN, bool WAIT, bool SO = false>
DLAP_DEV void mlp_fwd_body(const MlpJob& J, const MlpDims& D, char* smem, const int bx, const int gxw) {
  using Frag = typename P::Frag;
  Frag* lds = reinterpret_cast<Frag*>(smem);
  float* aux = aux_lds_ptr(smem, D);
  float* spp = pp_lds_ptr(smem, D);
  MLP_TS(0);
  const int wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  const int ntiles = (J.R + 31) >> 5;
  const int q = lane_id() >> 4, lane = lane_id();
  const int stride = gxw * nwaves;
  int tile = bx * nwaves + wave;
  int seen = 0;                          // WAIT: periods known to be published
  TileIn<P, KS1> cur, nxt;
  ZTile<WMB> zcur, znxt;                 // ZIN: layer-0 pre-activations instead of X rows
  AbPre<WMB> ab_cur, ab_nxt;
  int2 ti_ahead[2];                      // periods of the tile after next (for the abias prefetch)
  const bool mom = !SO && J.do_mom;
  // prologue: the step counter, the first tile's panel rows and keep words (both parity
  // halves: the step is not known yet) are all in flight with the weight staging
  const uint32_t stp = load_step(J);
  const bool pre = J.gbits && J.train && J.dropout > 0.f;   // keep words pre-generated (k_dropmask)
  constexpr int KWM = 4;                           // max SDF hidden layers (engine limit)
  uint32_t kw_cur[KWM], kw_nxt[KWM], kw_alt[KWM];
  auto issue_kw = [&](const DLAP_GLOBAL uint32_t* base, int t, uint32_t (&kw)[KWM], int nls) {
#pragma unroll
    for (int j = 0; j < KWM; ++j)
      kw[j] = j < nls ? base[((size_t)t * nls + j) * 64 + lane] : 0xFFFFFFFFu;
  };
  if (tile < ntiles) {
    if constexpr (ZIN) issue_ztile<WMB, false>(J, D, tile, zcur, J.do_sdf, mom);
    else issue_tile<P, KS1, false>(J, tile, cur);            // in flight during the staging
    if (mom && tile + stride < ntiles) issue_rowti(J, tile + stride, ti_ahead);
    if (pre) {
      issue_kw(gp(J.gbits), tile, kw_cur, D.nl_sdf);
      issue_kw(gp(J.gbits) + J.gb_half, tile, kw_alt, D.nl_sdf);
    }
  }
  stage_weights<P>(J, D, lds, aux, spp);
  MLP_TS(1);
  const DropCtx dc = drop_ctx(J, D, stp);
  const auto gbase = pre ? gp(J.gbits) + (size_t)(dc.step & 1u) * J.gb_half : nullptr;
  if (pre && (dc.step & 1u)) {
#pragma unroll
    for (int j = 0; j < KWM; ++j) kw_cur[j] = kw_alt[j];
  }
  if (mom && tile < ntiles) {
    if constexpr (ZIN) issue_abias<WMB>(J, zcur.ti, ab_cur);
    else issue_abias<WMB>(J, cur.ti, ab_cur);
  }
  const int pst = D.pp_lds_floats > 0 ? D.ppst : D.Dm;
  bool first = true;
  for (; tile < ntiles; tile += stride) {
    const int oz = opaque_zero();             // see bwd_sdf_body: no hoisted weight copies
    const Frag* ldt = lds + oz;
    const float* auxt = aux + oz;
    // depth tests made per tile from laundered copies: hoisted out of the loop they become
    // 64-bit lane masks that pin (and spill) SGPR pairs for the whole kernel
    MlpDims Dt = D;
    Dt.nl_sdf += oz;
    Dt.nl_mom += oz;
    if (tile + stride < ntiles) {
      if constexpr (ZIN) issue_ztile<WMB, false>(J, D, tile + stride, znxt, J.do_sdf, mom);
      else issue_tile<P, KS1, false>(J, tile + stride, nxt);
      if (pre) issue_kw(gbase, tile + stride, kw_nxt, Dt.nl_sdf);
      if (mom) {
        issue_abias<WMB>(J, ti_ahead, ab_nxt);             // periods known since last iteration
        if (tile + 2 * stride < ntiles) issue_rowti(J, tile + 2 * stride, ti_ahead);
      }
    }
    Frag xf[2][KS1];
    RowInfo ri;
    if constexpr (WAIT) {
      // the tile's last row (clamped to R - 1) has its largest period
      const int tl = __builtin_amdgcn_readlane(cur.ti[1].x, 15);
      seen = prog_wait(J.prog, J.prog_err, tl + 1, seen, J.prog_mode == 0, J.prog_limit);
      if (seen < 0) break;               // gave up: no writes from this wave (launch invalid)
    }
    if constexpr (ZIN) ri = finish_ztile<WMB>(J, tile, zcur);
    else if (WAIT && J.prog_mode != 0) ri = finish_tile<P, KS1, true, true>(J, D, tile, cur, xf, spp);
    else ri = finish_tile<P, KS1>(J, D, tile, cur, xf, spp);
    if (SO || J.do_sdf) {
      float w[2];
      uint32_t kw[4];
      if constexpr (SO) {
        DLAP_ASSERT(pre || !dc.on);
#pragma unroll
        for (int j = 0; j < 4; ++j) kw[j] = pre ? kw_cur[j] : 0xFFFFFFFFu;
      } else {
        sdf_keep_words(pre, kw_cur, dc, ri, Dt.nl_sdf, kw);
      }
      auto l0 = [&](f32x4 (&a)[2][4]) {
        if constexpr (ZIN) {
          if (D.pp_lds_floats > 0) zin_sdf0(zcur.zs, ri, spp, pst, auxt, D, a);
          else zin_sdf0(zcur.zs, ri, gp(J.pp), pst, auxt, D, a);
        } else {
          f32x4 init[2][4];
          bias_init<4>(auxt + D.a_sb, init);
          layer0<P, KS1, 4>(ldt, D.s_fwd0, xf, init, a);
        }
      };
      if (dc.on) sdf_forward_tile<P, true>(ldt, auxt, Dt, kw, l0, w);
      else sdf_forward_tile<P, false>(ldt, auxt, Dt, kw, l0, w);
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int r = tile * 32 + 16 * b + (lane & 15);
        if (q == 0 && r < J.R) gp(J.w_out)[r] = w[b];
      }
    }
    if (!SO && J.do_mom) {
      auto l0 = [&](f32x4 (&a)[2][WMB]) {
        if constexpr (ZIN) {
#pragma unroll
          for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int u = 0; u < WMB; ++u) a[b][u] = zcur.zm[b][u] + ab_cur.v[b][u];
        } else {
          layer0<P, KS1, WMB>(ldt, D.m_fwd0, xf, ab_cur.v, a);
        }
      };
      mom_forward_tile<P, WMB>(ldt, auxt, Dt, J, dc, ri, l0);
    }
    if constexpr (ZIN) zcur = znxt;
    else cur = nxt;
    ab_cur = ab_nxt;
#pragma unroll
    for (int j = 0; j < KWM; ++j) kw_cur[j] = kw_nxt[j];
    if (first) { MLP_TS(2); first = false; }
  }
  MLP_TS(3);
}

template <class P, int KS1, int WMB, bool ZIN, bool SO = false>
__global__ __launch_bounds__(256, DLAP_FWD_WPS) void k_mlp_fwd(const MlpJob* __restrict__ jobs, MlpDims D) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  mlp_fwd_body<P, KS1, WMB, ZIN, false, SO>(jobs[blockIdx.y], D, smem, blockIdx.x, gridDim.x);
}

// ============================== fused LSTM + training tower forward =======================
// The towers need the LSTM output of a row's period only, so the recurrence and the tower
// forward run as ONE launch: workgroup (0, job) runs the LSTM of that job's model on wave 0
// (lstm_gls_body, layer-0 input projections from k_proj), wave 1 publishes its progress --
// it polls the LDS step counter the recurrence bumps every 8 periods, copies the new outputs
// to J.out and release-stores the count to the job's global counter -- and every other
// workgroup runs the tower forward, waiting per tile for the periods of its rows. Tiles are
// visited in period order (tile index = bx * waves + wave, strided by the grid), so the
// towers trail the recurrence period by period instead of starting after it.
// Forward progress: each tower workgroup depends only on workgroup (0, its job). The engine
// launches the fused kernel only when its whole grid fits the device at once (occupancy query of
// the instantiation that runs, mlp_fwd_rnn_capacity), so on an otherwise idle device every
// workgroup is resident. Beside the evaluation branch of the pipelined epoch some workgroups may
// wait for CUs, but every kernel of that branch runs to completion without waiting on anything,
// so the CUs it holds are released and the fused grid becomes resident; only one fused (spinning)
// launch runs at a time. The spin is bounded anyway (prog_wait): a wait that gives up poisons the
// model instead of hanging the device.
DLAP_DEV void lstm_publish(const RnnJob& J, const ModelDesc* __restrict__ md, const float* sm, const int* sprog) {
  const int T = J.T, H = md->H, lane = threadIdx.x & 63;
  const float* shb = sm + gls_out_offset(T, H, md->nrnn);
  const auto out = gp(J.out);
  int done = 0;
  unsigned spins = 0;
  while (done < T) {
    const int p = __builtin_amdgcn_readfirstlane(__hip_atomic_load(sprog, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
    if (p <= done) {
      __builtin_amdgcn_s_sleep(1);
      // (never: the recurrence runs in the same workgroup and always finishes.) Giving up
      // publishes nothing more: the waiting tower waves then give up too, without writes.
      if (++spins > (1u << 22)) {
        if (lane == 0) atomicAdd(J.prog + 1, 1);
        return;
      }
      continue;
    }
    for (int i = done * H + lane; i < p * H; i += 64) out[i] = shb[i];
    // release: the outputs above are visible before the count (L2 written back, agent scope)
    if (lane == 0) __hip_atomic_store(J.prog, p, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    done = p;
  }
}

// ne > 0 (the pipelined phase-1/3 epoch): workgroups 1 .. ne of each job run the recurrences of
// that model's evaluation splits as well (rjobs[gridDim.y + job * ne + e], outputs flushed to
// their pp at the end; nothing waits for them inside this launch), so the evaluation branch
// starts at its tower forward right after this kernel instead of running its own LSTM launch
// beside the training chain (where it waited for CUs the spinning tower workgroups held).
// selfproj: the recurrences' layer-0 input projections are computed inside their workgroups
// (proj_into_lds on the spare waves, tile by tile ahead of the recurrence) instead of being staged
// from k_proj's output -- no k_proj launch before this one. (The train split's progress counter,
// which k_proj used to zero, is zeroed by the k_period_fwd that follows every fused forward.)
template <class P, int KS1, int WMB, int HM, bool DPPG, bool SO = false>
__global__ __launch_bounds__(256, DLAP_FWD_WPS) void k_mlp_fwd_rnn(const MlpJob* __restrict__ jobs, MlpDims D,
                                                                  const RnnJob* __restrict__ rjobs,
                                                                  const ModelDesc* __restrict__ md, int ne,
                                                                  int selfproj, int* esig) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = threadIdx.x >> 6;
  if (blockIdx.x >= 1 && (int)blockIdx.x <= ne) {
    const RnnJob& R = rjobs[gridDim.y + blockIdx.y * ne + (blockIdx.x - 1)];
    float* sx = reinterpret_cast<float*>(smem);
    if (md->nrnn == 0) return;
    // esig (the split epoch graphs): the recurrence wave, its outputs stored, releases them at
    // agent scope and counts itself -- the evaluation graph's first launch (k_wait_count) waits
    // for every evaluation recurrence of the launch
    auto signal = [&] {
      if (!esig) return;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(esig, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    if (selfproj) {
      int* ready = reinterpret_cast<int*>(sx + gls_ready_offset(R.T, md->H));
      for (int i = threadIdx.x; i < (R.T + 15) / 16; i += blockDim.x) ready[i] = 0;
      __syncthreads();
      // (timestamps 13-15: the last evaluation recurrence of model 0 -- the test split)
      const bool tse = blockIdx.y == 0 && (int)blockIdx.x == ne && jobs[0].gbits;
      if (tse && threadIdx.x == 0) g_mlp_ts[16] = wall_clock64();
      if (w == 0) { lstm_gls_body<HM, DPPG, false, false>(R, md, sx, nullptr, tse ? g_mlp_ts : nullptr, 16, ready); signal(); }
      else proj_into_lds(R, md, sx, ready, w - 1, 3, tse && w == 1 ? g_mlp_ts + 20 : nullptr);
      return;
    }
    const auto xg = gp(R.xg);
    const int n = R.T * 4 * md->H;
    for (int i = threadIdx.x; i < n; i += blockDim.x) sx[i] = xg[i];
    __syncthreads();
    if (w == 0) { lstm_gls_body<HM, DPPG, false, false>(R, md, sx, nullptr, nullptr, 0); signal(); }
    return;
  }
  if (blockIdx.x == 0) {
    __shared__ int s_prog;
    const RnnJob& R = rjobs[blockIdx.y];
    const bool tsm = blockIdx.y == 0 && jobs[0].gbits;
    float* sx = reinterpret_cast<float*>(smem);
    int* ready = selfproj ? reinterpret_cast<int*>(sx + gls_ready_offset(R.T, md->H)) : nullptr;
    if (threadIdx.x == 0) s_prog = 0;
    if (tsm && threadIdx.x == 0) g_mlp_ts[8] = wall_clock64();
    if (selfproj) {
      for (int i = threadIdx.x; i < (R.T + 15) / 16; i += blockDim.x) ready[i] = 0;
    } else {   // layer-0 input projections (k_proj) into the LDS staging area with all four waves
      const auto xg = gp(R.xg);
      const int n = md->nrnn > 0 ? R.T * 4 * md->H : 0;
      for (int i = threadIdx.x; i < n; i += blockDim.x) sx[i] = xg[i];
    }
    __syncthreads();
    if (w == 0) {
      lstm_gls_body<HM, DPPG, false, true>(R, md, sx, &s_prog, tsm ? g_mlp_ts : nullptr, 8, ready);
    } else if (w == 1) {
      lstm_publish(R, md, sx, &s_prog);
      if (tsm && threadIdx.x == 64) g_mlp_ts[12] = wall_clock64();
    } else if (selfproj) {
      proj_into_lds(R, md, sx, ready, w - 2, 2);
    }
    return;
  }
  mlp_fwd_body<P, KS1, WMB, false, true, SO>(jobs[blockIdx.y], D, smem, blockIdx.x - 1 - ne, gridDim.x - 1 - ne);
}

// ============================== wide evaluation forward ==================================
// Evaluation (no dropout, no backward) on the wide path: layer 0 of both towers is streamed
// from the panel rows inside the tower kernel -- k_proj0's loop with the layer-0 fragments
// staged in LDS next to the tower blob -- so the pre-activations never go through HBM (the
// z round trip is 2 x 320 B per row; an evaluation row is read once). grid (gx, jobs), 8 waves,
// one workgroup per CU (the layer-0 fragments take up to (4 + WMB) x KSX KiB of LDS). The
// next tile's first k-chunk is in flight while the tower runs on the current one.
// TRAIN: the training forward of the same kind -- dropout from the pre-generated keep words,
// and the layer-0 pre-activations stored to z (SDF blocks; the moment blocks too when
// J.store_mz, i.e. in phase 2) for the ZIN backward kernels.
template <int WMB, bool TRAIN>
__global__ __launch_bounds__(512, 1) void k_mlp_fwd_zx(const MlpJob* __restrict__ jobs, MlpDims D) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NU = 4 + WMB;
  const MlpJob& J = jobs[blockIdx.y];
  bf16x8* lds = reinterpret_cast<bf16x8*>(smem);
  float* aux = aux_lds_ptr(smem, D);
  float* spp = pp_lds_ptr(smem, D);
  bf16x8* lds0 = reinterpret_cast<bf16x8*>(smem + ((lds_bytes_of(D) + 15) & ~(size_t)15));
  const int lane = lane_id(), q = lane >> 4, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  const int KSX = D.KSX, rstride = D.KX >> 3;
  const int u0 = J.do_sdf ? 0 : 4, u1 = J.do_mom ? NU : 4;
  for (int i = threadIdx.x; i < (u1 - u0) * KSX * 64; i += blockDim.x) lds0[i] = gp(J.blob0)[u0 * KSX * 64 + i];
  const uint32_t stp = load_step(J);
  stage_weights<PrecBF16>(J, D, lds, aux, spp);           // (ends with the barrier)
  const DropCtx dc = drop_ctx(J, D, stp);
  const int ntiles = (J.R + 31) >> 5;
  const int nch = (KSX + 3) >> 2;
  const int stride = gridDim.x * nwaves;
  const int pst = D.pp_lds_floats > 0 ? D.ppst : D.Dm;
  int tile = blockIdx.x * nwaves + wave;
  if (tile >= ntiles) return;
  const bool pre = TRAIN && J.gbits && dc.on;
  const auto gbase = pre ? gp(J.gbits) + (size_t)(dc.step & 1u) * J.gb_half : nullptr;
  auto issue = [&](int tl, int ch, bf16x8 (&x)[2][4]) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int r = min(tl * 32 + 16 * b + (lane & 15), J.R - 1);
      const auto row = gp(J.X) + (size_t)r * rstride;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        // (unconditional: a k-step past KSX re-reads the last one, and the MFMAs skip it)
        x[b][s] = row[4 * min(4 * ch + s, KSX - 1) + q];
      }
    }
  };
  // panel chunks streamed two ahead: three register slots that rotate by unrolling the chunk loop
  // three times (a register copy of a slot whose load is in flight would wait for that load, so a
  // copy rotation keeps only the current chunk's MFMAs between a load and its use). Every chunk
  // load is issued -- past the wave's last tile it re-reads the last tile -- so the in-order load
  // counter is the same on every path. 16 KiB per wave in flight.
  bf16x8 xa[2][4], xb[2][4], xd[2][4];
  f32x4 acc[2][NU];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int u = 0; u < NU; ++u) acc[b][u] = zero4();
  int2 ti[2];
  issue_rowti(J, tile, ti);
  issue(tile, 0, xa);
  int ch = 0;
  auto advance = [&](int tl, int c, int& t2, int& c2) {
    t2 = tl; c2 = c + 1;
    if (c2 == nch) { c2 = 0; t2 += stride; }
  };
  int ntl, nc;
  advance(tile, ch, ntl, nc);
  bool more = ntl < ntiles;
  issue(min(ntl, ntiles - 1), nc, xb);
  // one chunk: the chunk two ahead goes into xn2, the current one (xc) runs; false after the last
  auto step = [&](const bf16x8 (&xc)[2][4], bf16x8 (&xn2)[2][4]) __attribute__((always_inline)) -> bool {
    int ntl2, nc2;
    advance(ntl, nc, ntl2, nc2);
    const bool more2 = more && ntl2 < ntiles;
    issue(min(ntl2, ntiles - 1), nc2, xn2);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int ks = 4 * ch + s;
      if (ks < KSX) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          if (u >= u0 && u < u1) {
            const bf16x8 w = lds0[((u - u0) * KSX + ks) * 64 + lane];
            acc[0][u] = mfma16(w, xc[0][s], acc[0][u]);
            acc[1][u] = mfma16(w, xc[1][s], acc[1][u]);
          }
        }
      }
    }
    if (nc == 0) {                                        // layer 0 of the tile is complete
      RowInfo ri;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int r = tile * 32 + 16 * b + (lane & 15);
        ri.t[b] = ti[b].x;
        ri.i[b] = ti[b].y;
        DLAP_ASSERT((unsigned)ri.t[b] < (unsigned)J.T && (unsigned)ri.i[b] < (unsigned)J.N);
        ri.dense[b] = r < J.R ? ti[b].x * J.N + ti[b].y : -1;
      }
      int2 tn[2];
      if (more) issue_rowti(J, ntl, tn);
      uint32_t kwp[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
      if constexpr (TRAIN) {
        const auto zt = gp(J.z_out) + (size_t)tile * D.zc * 64 + lane;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
#pragma unroll
          for (int u = 0; u < 4; ++u) zt[(4 * b + u) * 64] = acc[b][u];
          if (J.store_mz) {
#pragma unroll
            for (int u = 0; u < WMB; ++u) zt[(8 + WMB * b + u) * 64] = acc[b][4 + u];
          }
        }
        if (pre) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            kwp[j] = j < D.nl_sdf ? gbase[((size_t)tile * D.nl_sdf + j) * 64 + lane] : 0xFFFFFFFFu;
        }
      }
      if (J.do_sdf) {
        f32x4 zs[2][4];
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int u = 0; u < 4; ++u) zs[b][u] = acc[b][u];
        auto l0 = [&](f32x4 (&a)[2][4]) {
          if (D.pp_lds_floats > 0) zin_sdf0(zs, ri, spp, pst, aux, D, a);
          else zin_sdf0(zs, ri, gp(J.pp), pst, aux, D, a);
        };
        uint32_t kw[4];
        sdf_keep_words(pre, kwp, dc, ri, D.nl_sdf, kw);
        float w[2];
        if (dc.on) sdf_forward_tile<PrecBF16, true>(lds, aux, D, kw, l0, w);
        else sdf_forward_tile<PrecBF16, false>(lds, aux, D, kw, l0, w);
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int r = tile * 32 + 16 * b + (lane & 15);
          if (q == 0 && r < J.R) gp(J.w_out)[r] = w[b];
        }
      }
      if (J.do_mom) {
        AbPre<WMB> ab;
        issue_abias<WMB>(J, ti, ab);
        auto l0m = [&](f32x4 (&a)[2][WMB]) {
#pragma unroll
          for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int u = 0; u < WMB; ++u) a[b][u] = acc[b][4 + u] + ab.v[b][u];
        };
        mom_forward_tile<PrecBF16, WMB>(lds, aux, D, J, dc, ri, l0m);
      }
      // drain the vector-memory counter once per tile: the tile's stores (w_out, z) sit between
      // loads and their uses in the vmcnt order, and a store may complete before an older load
      // (measured: without this wait the evaluation outputs of the unrolled loop were
      // nondeterministic, tools/wide_det_probe.py); the chunk prefetch inside a tile is untouched
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int b = 0; b < 2; ++b) {
#pragma unroll
        for (int u = 0; u < NU; ++u) acc[b][u] = zero4();
        if (more) ti[b] = tn[b];
      }
    }
    if (!more) return false;
    tile = ntl;
    ch = nc;
    ntl = ntl2;
    nc = nc2;
    more = more2;
    return true;
  };
  while (step(xa, xd) && step(xb, xa) && step(xd, xb)) {
  }
}

// ============================== backward =================================================
template <class P, int UB>
DLAP_DEV void to_rows_k(const typename P::Frag (&pf)[2][(UB + 1) / 2], int blk, const typename P::Frag& s0,
                        const typename P::Frag& s1, typename P::Frag& out) {
  const typename P::Frag sel = (blk & 1) ? s1 : s0;
  out = P::pack(P::mma(pf[0][blk >> 1], sel, zero4()), P::mma(pf[1][blk >> 1], sel, zero4()));
}

template <class P>
DLAP_DEV void x_rows_k(const typename P::Frag& x0, const typename P::Frag& x1, int blk,
                       const typename P::Frag& s0, const typename P::Frag& s1, typename P::Frag& out) {
  const typename P::Frag sel = (blk & 1) ? s1 : s0;
  out = P::pack(P::mma(x0, sel, zero4()), P::mma(x1, sel, zero4()));
}

// Fine slabs per workgroup: FPW = 1 compiled in (the one-slab launch: no slab loop state in the
// register budget of the two-waves-per-SIMD kernel, ~2% faster at 600x3000x46) or 0 = J.fpw
#define BWD_FPW(J) (FPW ? FPW : (J).fpw)

// One slab per workgroup: zero an LDS image (reusing the weight staging area), let the
// waves add into it one after another (fixed order = deterministic), then store it.
DLAP_DEV float* wg_slab_begin(char* smem, int slab_stride) {
  __syncthreads();   // every wave is done with the staged weights
  float* red = reinterpret_cast<float*>(smem);
  for (int i = threadIdx.x; i < slab_stride; i += blockDim.x) red[i] = 0.f;
  __syncthreads();
  return red;
}
// LDS image of a slab (bank-conflict-free wave adds): the global slab layout is natural --
// gradient tile t element (o, i) at t*4096 + 64 o + i, then the extra rows (per-layer bias rows
// of 64, the output row, the output bias) -- but in LDS
//   * tile elements store i with bit 4 flipped for odd o>>2: a wave adds (o = 16u + 4q + r,
//     i = 16v + n) with lane n + 16q, so the lanes of q and q+1 (one 32-lane group of
//     ds_read_b32 / ds_write_b32, bank = dword mod 32) hit opposite bank halves instead of the
//     same 16 banks (2-way);
//   * bias row j stores column c at (c + 5 j) mod 64, so the up-to-6 layer lanes (n = j) of a
//     group are 5 banks apart instead of all on one bank (16-way was ~2/3 of the 832 conflicts
//     per wave measured on k_mlp_bwd_sdf, profiles/r3_final_pmc_summary.txt).
template <int TPS>
DLAP_DEV int slab_lds(int e) {
  if (e < TPS * 4096) return e ^ ((((e >> 6) >> 2) & 1) << 4);
  const int x = e - TPS * 4096;
  if (x < DLAP_MAXL * 64) {
    const int j = x >> 6;
    return TPS * 4096 + (j << 6) + (((x & 63) + 5 * j) & 63);
  }
  return e;
}

// Fine slab k (of J.fpw) of this workgroup is complete in `red` (after the wave loop's final
// barrier). fpw == 1: store it as fine slab blockIdx.x of the slice. Else accumulate it, in
// order, into the workgroup's coarse image in LDS right after `red` (same swizzled layout, each
// thread adds only its own elements): ((s0 + s1) + s2) + s3 -- exactly the grouping k_finalize
// applies to stored fine slabs, so either launch shape gives the same gradient bits -- and store
// the coarse slab after the last one. (A global read-modify-write per fine slab cost ~20 us per
// flush at G = 9: the loads of the loop serialise behind the stores they may alias.)
template <int TPS, int FPW>
DLAP_DEV void wg_slab_finish(const MlpJob& J, float* red, int slab_stride, int k) {
  const int fpw = BWD_FPW(J);
  const int nst = J.nslab / fpw;                   // slabs stored per slice
  const auto slab = gp(J.slab) + (size_t)(J.slab_base + blockIdx.z * nst + blockIdx.x) * slab_stride;
  if (fpw == 1) {
    for (int i = threadIdx.x; i < slab_stride; i += blockDim.x) slab[i] = red[slab_lds<TPS>(i)];
    return;
  }
  float* coarse = red + slab_stride;
  if (k == 0) {
    for (int i = threadIdx.x; i < slab_stride; i += blockDim.x) coarse[i] = red[i];
  } else {
    for (int i = threadIdx.x; i < slab_stride; i += blockDim.x) coarse[i] = coarse[i] + red[i];
  }
  if (k + 1 < fpw) return;
  __syncthreads();
  for (int i = threadIdx.x; i < slab_stride; i += blockDim.x) slab[i] = coarse[slab_lds<TPS>(i)];
}

// SDF backward. NL = number of hidden (MFMA) layers, all 64 wide.
// The forward of the tile is recomputed from the panel (with this step's keep words, the train
// blob: dropout scale folded into the weights), the ReLU'/dropout gates come from the recomputed
// packed activations, and every dz goes straight into packed operand fragments.
// ZIN (wide path): layer 0 is recomputed from z, its weight gradient is left to k_wgrad0: the
// kernel stores the layer-0 dz as rows-as-k fragments instead (J.dz_out [tile][4][64]).
// TLC: the layer of this slice's gradient tile when it is known at compile time (TPS = 1, one
// instantiation per layer, selected from blockIdx.z); -2: TPS = 2 on a two-tile tower (tile t
// is layer t, one slice), so every gradient MFMA is unconditional and the accumulators stay
// in place across the tile loop; else -1 (runtime tile map). A slice of layer TLC > 0 stops
// its backward chain at that layer and leaves the bias / output-layer / per-period input
// gradients to slice 0, so its live state (and register budget) is that of its own role.
template <class P, int KS1, int NL, int TPS, bool ZIN, int TLC, int FPW>
DLAP_DEV void bwd_sdf_body(const MlpJob& J, const MlpDims& D, int slab_stride, char* smem, int slice, int C0,
                           int red_off) {
  using Frag = typename P::Frag;
  Frag* lds = reinterpret_cast<Frag*>(smem);
  float* aux = aux_lds_ptr(smem, D);
  float* spp = pp_lds_ptr(smem, D);
  // fine slab image: over the staging area (one fine slab per workgroup) or, walking several,
  // beyond it (red_off > 0), so the staged weights stay valid for the next fine slab
  char* const sred = smem + red_off;
  const int lane = lane_id(), q = lane >> 4, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  const int ntiles = (J.R + 31) >> 5;
  const bool s0 = TLC <= 0 && slice == 0;      // the slice that owns the extra gradients (-2: slice 0)
  constexpr int JLO = TLC > 0 ? TLC : 0;        // lowest layer the backward chain reaches
  const Frag selP0 = make_sel<P>(true, 0), selP1 = make_sel<P>(true, 1);
  const Frag selN0 = make_sel<P>(false, 0), selN1 = make_sel<P>(false, 1);
  const int pst = D.pp_lds_floats > 0 ? D.ppst : D.Dm;
  int tl[TPS], tc[TPS];
#pragma unroll
  for (int t = 0; t < TPS; ++t) {
    const int tid = slice * TPS + t;
    tl[t] = TLC == -2 ? t : TLC >= 0 ? TLC : (tid < C0 ? 0 : tid - C0 + 1);
    tc[t] = (TLC == -2 || TLC > 0) ? 0 : (tid < C0 ? tid : 0);
  }
  // fine slab vs = blockIdx.x * fpw + k owns tiles vs * waves + wave, strided by nslab * waves:
  // the partition (and so every fp32 partial) depends on R only, never on the launch grid
  const int stride = J.nslab * nwaves;
  const uint32_t stp = load_step(J);
  const bool pre = J.gbits && J.train && J.dropout > 0.f;   // keep words of this step (k_dropmask)
  for (int kf = 0; kf < BWD_FPW(J); ++kf) {
  if (kf) __syncthreads();                      // the previous slab's LDS reads are done
  f32x4 dW[TPS][4][4];
#pragma unroll
  for (int t = 0; t < TPS; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) dW[t][u][v] = zero4();
  f32x4 gbias[4], gwo[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) { gbias[u] = zero4(); gwo[u] = zero4(); }
  float gbo = 0.f;
  int tile = (blockIdx.x * BWD_FPW(J) + kf) * nwaves + wave;
  TileIn<P, KS1> cur, nxt;
  ZTile<1> zcur, znxt;
  // prologue as k_mlp_fwd: step, first tile and its keep words of both parities in flight with
  // the staging (re-staged per fine slab: the slab reduction reuses the staging area)
  uint32_t kw_cur[NL], kw_nxt[NL], kw_alt[NL];
  if (tile < ntiles) {
    if constexpr (ZIN) issue_ztile<1, true>(J, D, tile, zcur, true, false);
    else issue_tile<P, KS1, true>(J, tile, cur);
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      kw_cur[j] = pre ? *gp32(J.gbits, (uint32_t)((tile * NL + j) * 64 + lane)) : 0xFFFFFFFFu;
      kw_alt[j] = pre ? *gp32(J.gbits, (uint32_t)(J.gb_half + (tile * NL + j) * 64 + lane)) : 0xFFFFFFFFu;
    }
  }
  if (kf == 0) stage_weights<P>(J, D, lds, aux, spp);   // first tile's loads are already in flight
  const DropCtx dc = drop_ctx(J, D, stp);
  const auto gbase = pre ? gp(J.gbits) + (size_t)(dc.step & 1u) * J.gb_half : nullptr;
  if (dc.step & 1u) {
#pragma unroll
    for (int j = 0; j < NL; ++j) kw_cur[j] = kw_alt[j];
  }
  for (; tile < ntiles; tile += stride) {
    // LDS base laundered per tile: keeps the compiler from hoisting every weight fragment and
    // bias of the staged blob out of the loop into registers (~150 VGPRs at this depth)
    const int oz = opaque_zero();
    const Frag* ldt = lds + oz;
    const float* auxt = aux + oz;
    if (tile + stride < ntiles) {
      if constexpr (ZIN) issue_ztile<1, true>(J, D, tile + stride, znxt, true, false);
      else issue_tile<P, KS1, true>(J, tile + stride, nxt);
#pragma unroll
      for (int j = 0; j < NL; ++j)
        kw_nxt[j] = pre ? *at32(gbase, (uint32_t)(((tile + stride) * NL + j) * 64 + lane)) : 0xFFFFFFFFu;
    }
    Frag xf[2][KS1];
    RowInfo ri;
    if constexpr (ZIN) ri = finish_ztile<1>(J, tile, zcur);
    else ri = finish_tile<P, KS1>(J, D, tile, cur, xf, spp);
    // SDF backward launches always read pre-generated keep words (k_dropmask runs ahead of every
    // phase-1/3 step that trains with dropout), so no hash path is compiled into the tile loop
    DLAP_ASSERT(pre || !dc.on);
    uint32_t kw[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) kw[j] = kw_cur[j];
    // ---- forward recompute: packed activations of every hidden layer ----
    Frag act[NL][2][2];
    f32x4 a[2][4];
    if constexpr (ZIN) {
      if (D.pp_lds_floats > 0) zin_sdf0(zcur.zs, ri, spp, pst, auxt, D, a);
      else zin_sdf0(zcur.zs, ri, gp(J.pp), pst, auxt, D, a);
    } else {
      f32x4 init[2][4];
      bias_init<4>(auxt + D.a_sb, init);
      layer0<P, KS1, 4>(ldt, D.s_fwd0, xf, init, a);
    }
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      if (j > 0) layer_chain<P, 4, 2>(ldt, D.s_fwd + (j - 1) * 8, act[j - 1], a, auxt + D.a_sb + 64 * j);
      act_tile_rt<P, 4>(a, dc.on, kw[j], act[j]);
    }
    // ---- output layer: w = wo' . act + bo (wo' = wo / (1 - p): train aux) ----
    float dwr[2];
    if constexpr (ZIN) { dwr[0] = zcur.dw[0]; dwr[1] = zcur.dw[1]; }
    else { dwr[0] = cur.dw[0]; dwr[1] = cur.dw[1]; }
    Frag dzf[2][2];
    {
      const float* wo = auxt + D.a_wo;
      f32x4 t[2][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f32x4 ww = ld4(wo + 16 * u + 4 * q);
        t[0][u] = dwr[0] * ww;
        t[1][u] = dwr[1] * ww;
      }
      gate_tile<P, 4>(t, act[NL - 1], dzf);
    }
    if (s0) {
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          f32x4 lo, hi;
          P::unpack(act[NL - 1][b][s], lo, hi);
          gwo[2 * s] += dwr[b] * lo;
          gwo[2 * s + 1] += dwr[b] * hi;
        }
      if (q == 0) gbo += dwr[0] + dwr[1];
    }
    // ---- backward chain ----
#pragma unroll
    for (int j = NL - 1; j >= 0; --j) {
      if (j < JLO) break;
      Frag dzN[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) to_rows_k<P, 4>(dzf, u, selP0, selP1, dzN[u]);
      if (s0) {
        const Frag oh = make_onehot<P>(j);
#pragma unroll
        for (int u = 0; u < 4; ++u) gbias[u] = P::mma(dzN[u], oh, gbias[u]);
      }
      if constexpr (ZIN) {
        if (j == 0 && s0) {                         // layer-0 dz for k_wgrad0
          const auto dzo = gp(reinterpret_cast<Frag*>(J.dz_out)) + (size_t)tile * 4 * 64 + lane;
#pragma unroll
          for (int u = 0; u < 4; ++u) dzo[u * 64] = dzN[u];
        }
      }
#pragma unroll
      for (int t = 0; t < TPS; ++t) {
        if (tl[t] == j) {
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            Frag aN = P::zero();
            if (j == 0) {
              const int blk = 4 * tc[t] + v;
              if constexpr (!ZIN) {
                Frag x0 = P::zero(), x1 = P::zero();
#pragma unroll
                for (int s = 0; s < KS1; ++s)
                  if (s == (blk >> 1)) { x0 = xf[0][s]; x1 = xf[1][s]; }
                x_rows_k<P>(x0, x1, blk, selN0, selN1, aN);
              } else {
                if (16 * blk >= D.Dm) continue;             // wave-uniform: no columns here
                Frag x0, x1;
                if (D.pp_lds_floats > 0) {
                  x0 = pp_xfrag<P>(spp, pst, ri.t[0], blk >> 1, D); x1 = pp_xfrag<P>(spp, pst, ri.t[1], blk >> 1, D);
                } else {
                  x0 = pp_xfrag<P>(gp(J.pp), pst, ri.t[0], blk >> 1, D); x1 = pp_xfrag<P>(gp(J.pp), pst, ri.t[1], blk >> 1, D);
                }
                x_rows_k<P>(x0, x1, blk, selN0, selN1, aN);
              }
            } else {
              to_rows_k<P, 4>(act[j > 0 ? j - 1 : 0], v, selP0, selP1, aN);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) dW[t][u][v] = P::mma(dzN[u], aN, dW[t][u][v]);
          }
        }
      }
      if (j > JLO) {
        f32x4 da[2][4];
        layer_chain<P, 4, 2>(ldt, D.s_bwd + (j - 1) * 8, dzf, da);
        gate_tile<P, 4>(da, act[j > 0 ? j - 1 : 0], dzf);
      } else if (j == 0 && D.nrnn > 0 && s0) {
        // dL/d(per-period input d) per row = sum_out W0[out][F + d] * dz0[out][row]: one MFMA
        // chain per 16 inputs with the packed W0[:, F:F+Dm]^T fragments
        for (int ub = 0; ub < D.ubpp; ++ub) {
          f32x4 c0 = zero4(), c1 = zero4();
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const Frag w = ldsf(ldt, D.s_upp + 2 * ub + s);
            c0 = P::mma(w, dzf[0][s], c0);
            c1 = P::mma(w, dzf[1][s], c1);
          }
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int row = tile * 32 + 16 * b + (lane & 15);
            const f32x4 c = b ? c1 : c0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int d = 16 * ub + 4 * q + r;
              if (d < D.Dm && row < J.R) *gp32(J.u_out, (uint32_t)(row * D.Dm + d)) = c[r];
            }
          }
        }
      }
    }
    if constexpr (ZIN) zcur = znxt;
    else cur = nxt;
#pragma unroll
    for (int j = 0; j < NL; ++j) kw_cur[j] = kw_nxt[j];
  }
  // ---- workgroup slab: waves add their partials into LDS in a fixed order ----
  float* red = wg_slab_begin(sred, slab_stride);
  for (int w = 0; w < nwaves; ++w) {
    if (wave == w) {
#pragma unroll
      for (int t = 0; t < TPS; ++t)
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int v = 0; v < 4; ++v)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              red[t * 4096 + (16 * u + 4 * q + r) * 64 + ((16 * v + (lane & 15)) ^ ((q & 1) << 4))] += dW[t][u][v][r];
      if (s0) {
        float* ex = red + TPS * 4096;
        const int jl = lane & 15;
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (jl < DLAP_MAXL) ex[jl * 64 + ((16 * u + 4 * q + r + 5 * jl) & 63)] += gbias[u][r];
            float v = gwo[u][r];
            v += __shfl_xor(v, 1, 64); v += __shfl_xor(v, 2, 64);
            v += __shfl_xor(v, 4, 64); v += __shfl_xor(v, 8, 64);
            if ((lane & 15) == 0) ex[DLAP_MAXL * 64 + 16 * u + 4 * q + r] += v;
          }
        const float sb = wave_sum(gbo);
        if (lane == 0) ex[DLAP_MAXL * 64 + 64] += sb;
      }
    }
    __syncthreads();
  }
  wg_slab_finish<TPS, FPW>(J, red, slab_stride, kf);
  }
}

template <class P, int KS1, int NL, int TPS, bool ZIN, int FPW>
__global__ __launch_bounds__(256, TPS == 1 ? DLAP_BWD1_WPS : 1) void k_mlp_bwd_sdf(const MlpJob* __restrict__ jobs, MlpDims D,
                                                        int slab_stride, int red_off) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const MlpJob& J = jobs[blockIdx.y];
  const int slice = blockIdx.z;
  // 64-column chunks of layer 0 with a gradient tile: the X chunks (fused) or, on the wide
  // path, only the per-period input columns (the X columns are k_wgrad0's)
  const int C0 = ZIN ? (D.Dm + 63) / 64 : KS1 / 2;
  if constexpr (TPS == 1) {
    const int tl = slice < C0 ? 0 : slice - C0 + 1;     // block-uniform: one role per slice
    if (tl == 0) bwd_sdf_body<P, KS1, NL, 1, ZIN, 0, FPW>(J, D, slab_stride, smem, slice, C0, red_off);
    if constexpr (NL > 1) if (tl == 1) bwd_sdf_body<P, KS1, NL, 1, ZIN, 1, FPW>(J, D, slab_stride, smem, slice, C0, red_off);
    if constexpr (NL > 2) if (tl == 2) bwd_sdf_body<P, KS1, NL, 1, ZIN, 2, FPW>(J, D, slab_stride, smem, slice, C0, red_off);
    if constexpr (NL > 3) if (tl == 3) bwd_sdf_body<P, KS1, NL, 1, ZIN, 3, FPW>(J, D, slab_stride, smem, slice, C0, red_off);
  } else if (TPS == 2 && C0 == 1) {     // the engine's TPS = 2 case: tiles (layer 0, layer 1)
    bwd_sdf_body<P, KS1, NL, TPS, ZIN, -2, FPW>(J, D, slab_stride, smem, slice, C0, red_off);
  } else {
    bwd_sdf_body<P, KS1, NL, TPS, ZIN, -1, FPW>(J, D, slab_stride, smem, slice, C0, red_off);
  }
}


// Moment backward (phase 2). NLM MFMA layers of WM = 16*WMB units; tanh on the last. Hidden
// layers' keep words are hashed as in the forward; gates from the recomputed activations.
// ZIN: as k_mlp_bwd_sdf (layer 0 from z, layer-0 dz stored as J.dz_out [tile][WMB][64]).
template <class P, int KS1, int WMB, int NLM, int TPS, bool ZIN>
__global__ __launch_bounds__(256, 1) void k_mlp_bwd_mom(const MlpJob* __restrict__ jobs, MlpDims D,
                                                        int slab_stride, int red_off) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KSM = (WMB + 1) / 2;
  using Frag = typename P::Frag;
  const MlpJob& J = jobs[blockIdx.y];
  Frag* lds = reinterpret_cast<Frag*>(smem);
  float* aux = aux_lds_ptr(smem, D);
  char* const sred = smem + red_off;         // fine slab image (see bwd_sdf_body)
  const int lane = lane_id(), q = lane >> 4, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  const int ntiles = (J.R + 31) >> 5;
  const int slice = blockIdx.z;
  constexpr int C0 = ZIN ? 0 : KS1 / 2;
  const Frag selP0 = make_sel<P>(true, 0), selP1 = make_sel<P>(true, 1);
  const Frag selN0 = make_sel<P>(false, 0), selN1 = make_sel<P>(false, 1);
  int tl[TPS], tc[TPS];
#pragma unroll
  for (int t = 0; t < TPS; ++t) {
    const int tid = slice * TPS + t;
    tl[t] = tid < C0 ? 0 : tid - C0 + 1;
    tc[t] = tid < C0 ? tid : 0;
  }
  // fine slabs as k_mlp_bwd_sdf (partition of the rows by R only)
  const int stride = J.nslab * nwaves;
  for (int kf = 0; kf < J.fpw; ++kf) {
  if (kf) __syncthreads();
  f32x4 dW[TPS][WMB][4];
#pragma unroll
  for (int t = 0; t < TPS; ++t)
#pragma unroll
    for (int u = 0; u < WMB; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) dW[t][u][v] = zero4();
  f32x4 gbias[WMB];
#pragma unroll
  for (int u = 0; u < WMB; ++u) gbias[u] = zero4();
  int tile = (blockIdx.x * J.fpw + kf) * nwaves + wave;
  TileIn<P, KS1> cur, nxt;
  ZTile<WMB> zcur, znxt;
  AbPre<WMB> ab_cur, ab_nxt;
  int2 ti_ahead[2];
  if (tile < ntiles) {
    if constexpr (ZIN) issue_ztile<WMB, false>(J, D, tile, zcur, false, true);
    else issue_tile<P, KS1, false>(J, tile, cur);
    if (tile + stride < ntiles) issue_rowti(J, tile + stride, ti_ahead);
  }
  const uint32_t stp = load_step(J);
  if (kf == 0) stage_weights<P>(J, D, lds, aux);
  const DropCtx dc = drop_ctx(J, D, stp);
  if (tile < ntiles) {
    if constexpr (ZIN) issue_abias<WMB>(J, zcur.ti, ab_cur);
    else issue_abias<WMB>(J, cur.ti, ab_cur);
  }
  for (; tile < ntiles; tile += stride) {
    const int oz = opaque_zero();             // see bwd_sdf_body: no hoisted weight copies
    const Frag* ldt = lds + oz;
    const float* auxt = aux + oz;
    if (tile + stride < ntiles) {
      if constexpr (ZIN) issue_ztile<WMB, false>(J, D, tile + stride, znxt, false, true);
      else issue_tile<P, KS1, false>(J, tile + stride, nxt);
      issue_abias<WMB>(J, ti_ahead, ab_nxt);
      if (tile + 2 * stride < ntiles) issue_rowti(J, tile + 2 * stride, ti_ahead);
    }
    Frag xf[2][KS1];
    RowInfo ri;
    if constexpr (ZIN) ri = finish_ztile<WMB>(J, tile, zcur);
    else ri = finish_tile<P, KS1, false>(J, D, tile, cur, xf);   // moment tower: no per-period cols
    Frag act[NLM][2][KSM];
    f32x4 a[2][WMB];
    if constexpr (ZIN) {
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int u = 0; u < WMB; ++u) a[b][u] = zcur.zm[b][u] + ab_cur.v[b][u];
    } else {
      layer0<P, KS1, WMB>(ldt, D.m_fwd0, xf, ab_cur.v, a);
    }
    f32x4 dz[2][WMB];
#pragma unroll
    for (int j = 0; j < NLM; ++j) {
      if (j > 0) layer_chain<P, WMB, KSM>(ldt, D.m_fwd + (j - 1) * WMB * KSM, act[j - 1], a, auxt + D.a_mb + 64 * j);
      if (j + 1 < NLM) {
        const uint32_t kw = dc.on ? hash_keep<WMB>(dc, 16 + j, ri) : 0xFFFFFFFFu;
        act_tile_rt<P, WMB>(a, dc.on, kw, act[j]);
      } else {
        // h = tanh(z); dz = dh (1 - h^2), dh = dE[i][k] R SDF_t / T_i (the moment loss), or an
        // external dL/dh (module API: a caller's loss of the moments)
        const bool ext = J.dh_ext != nullptr;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int d = ri.dense[b];
          const float cst = (d >= 0 && !ext) ? gp(J.Rm)[d] * gp(J.sdfv)[ri.t[b]] * gp(J.invT)[ri.i[b]] : 0.f;
          const auto de = ext ? gp(J.dh_ext) + (size_t)(d >= 0 ? d : 0) * D.K : gp(J.dE) + (size_t)ri.i[b] * D.K;
#pragma unroll
          for (int u = 0; u < WMB; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int k = 16 * u + 4 * q + r;
              const float h = tanhf(a[b][u][r]);
              const float g = (d >= 0 && k < D.K) ? (ext ? de[k] : de[k] * cst) : 0.f;
              dz[b][u][r] = g * (1.f - h * h);
            }
        }
      }
    }
    Frag dzf[2][KSM];
    pack_blocks<P, WMB>(dz, dzf);
#pragma unroll
    for (int j = NLM - 1; j >= 0; --j) {
      Frag dzN[WMB];
#pragma unroll
      for (int u = 0; u < WMB; ++u) to_rows_k<P, WMB>(dzf, u, selP0, selP1, dzN[u]);
      if (slice == 0 && j > 0) {
        const Frag oh = make_onehot<P>(j);
#pragma unroll
        for (int u = 0; u < WMB; ++u) gbias[u] = P::mma(dzN[u], oh, gbias[u]);
      }
      if constexpr (ZIN) {
        if (j == 0 && slice == 0) {                 // layer-0 dz for k_wgrad0
          const auto dzo = gp(reinterpret_cast<Frag*>(J.dz_out)) + (size_t)tile * WMB * 64 + lane;
#pragma unroll
          for (int u = 0; u < WMB; ++u) dzo[u * 64] = dzN[u];
        }
      }
#pragma unroll
      for (int t = 0; t < TPS; ++t) {
        if (tl[t] == j) {
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            if (j > 0 && v >= WMB) continue;
            Frag aN = P::zero();
            if (j == 0) {
              if constexpr (!ZIN) {
                const int blk = 4 * tc[t] + v;
                Frag x0 = P::zero(), x1 = P::zero();
#pragma unroll
                for (int s = 0; s < KS1; ++s)
                  if (s == (blk >> 1)) { x0 = xf[0][s]; x1 = xf[1][s]; }
                x_rows_k<P>(x0, x1, blk, selN0, selN1, aN);
              }
            } else {
              to_rows_k<P, WMB>(act[j > 0 ? j - 1 : 0], v, selP0, selP1, aN);
            }
#pragma unroll
            for (int u = 0; u < WMB; ++u) dW[t][u][v] = P::mma(dzN[u], aN, dW[t][u][v]);
          }
        }
      }
      if (j > 0) {
        f32x4 da[2][WMB];
        layer_chain<P, WMB, KSM>(ldt, D.m_bwd + (j - 1) * WMB * KSM, dzf, da);
        gate_tile<P, WMB>(da, act[j > 0 ? j - 1 : 0], dzf);
      } else if (slice == 0) {
        // dL/d(layer-0 pre-activation) per row for the macro-column / bias gradients: fp32 when
        // layer 0 is the tanh layer, else the packed dz0 unpacked (the values the weight-gradient
        // MFMAs used)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int row = tile * 32 + 16 * b + (lane & 15);
          if (row < J.R) {
#pragma unroll
            for (int s = 0; s < KSM; ++s) {
              f32x4 lo, hi;
              if (NLM == 1) { lo = dz[b][2 * s]; hi = dz[b][(2 * s + 1) % WMB]; }
              else P::unpack(dzf[b][s], lo, hi);
              *reinterpret_cast<f32x4*>(gp(J.v_out) + (size_t)row * 64 + 32 * s + 4 * q) = lo;
              if (2 * s + 1 < WMB) *reinterpret_cast<f32x4*>(gp(J.v_out) + (size_t)row * 64 + 32 * s + 16 + 4 * q) = hi;
            }
          }
        }
      }
    }
    if constexpr (ZIN) zcur = znxt;
    else cur = nxt;
    ab_cur = ab_nxt;
  }
  float* red = wg_slab_begin(sred, slab_stride);
  for (int w = 0; w < nwaves; ++w) {
    if (wave == w) {
#pragma unroll
      for (int t = 0; t < TPS; ++t)
#pragma unroll
        for (int u = 0; u < WMB; ++u)
#pragma unroll
          for (int v = 0; v < 4; ++v)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              red[t * 4096 + (16 * u + 4 * q + r) * 64 + ((16 * v + (lane & 15)) ^ ((q & 1) << 4))] += dW[t][u][v][r];
      if (slice == 0) {
        float* ex = red + TPS * 4096;
        const int jl = lane & 15;
#pragma unroll
        for (int u = 0; u < WMB; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (jl < DLAP_MAXL) ex[jl * 64 + ((16 * u + 4 * q + r + 5 * jl) & 63)] += gbias[u][r];
      }
    }
    __syncthreads();
  }
  wg_slab_finish<TPS, 0>(J, red, slab_stride, kf);
  }
}

// ============================== dropout keep-mask generator ===========================
// Keep words of every (tile, SDF layer, lane) for the dropout step *step + step_offset*, in
// that step's parity half of gbits (split layout, keep_word). Generating them here lets the
// next step's masks be produced on an idle branch of the epoch graph while the serial LSTM
// kernels run; the training forward and the backward of that step both read them.
__global__ __launch_bounds__(256) void k_dropmask(const MlpJob* __restrict__ jobs, MlpDims D, int step_offset) {
  const MlpJob& J = jobs[blockIdx.y];
  const int ntiles = (J.R + 31) >> 5;
  const int gid = blockIdx.x * 256 + threadIdx.x;
  const int tile = gid >> 6, lane = gid & 63, q = lane >> 4;
  if (tile >= ntiles) return;
  const uint32_t step = (J.step ? (uint32_t)*gp(J.step) : 0u) + (uint32_t)step_offset;
  if (!(J.dropout > 0.f)) return;        // (no keep words: this model's towers do not read them)
  const uint32_t thr16 = (uint32_t)(J.dropout * 65536.f + 0.5f);
  uint32_t rowmix[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int r = tile * 32 + 16 * b + (lane & 15);
    const int2 ti = gp(J.rowti)[min(r, J.R - 1)];
    // rows beyond R hash as dense row -1, as the towers do (their words are never used)
    rowmix[b] = row_mix(r < J.R ? (uint32_t)(ti.x * J.N + ti.y) : 0xFFFFFFFFu);
  }
  const auto dst = gp(const_cast<uint32_t*>(J.gbits)) + (size_t)(step & 1u) * J.gb_half + (size_t)tile * D.nl_sdf * 64 + lane;
  for (int j = 0; j < D.nl_sdf; ++j) dst[64 * j] = keep_word<4>(dropout_key(J.seed, step, j), rowmix, thr16, q);
}

void launch_dropmask(const MlpJob* jobs, int njobs, int ntiles, const MlpDims& D, int step_offset,
                     hipStream_t st) {
  hipLaunchKernelGGL(k_dropmask, dim3((ntiles * 64 + 255) / 256, njobs), dim3(256), 0, st, jobs, D,
                     step_offset);
  HIP_OK(hipGetLastError());
}

// ---- host launchers -------------------------------------------------------------------
size_t mlp_lds_bytes(const MlpDims& D) { return lds_bytes_of(D); }
// backward LDS: the staging area, reused by the fine slab image when a workgroup walks one
// fine slab; walking several (fpw > 1) the fine and coarse images go beyond it (red_off), so
// the weights are staged once
static size_t bwd_red_off(const MlpDims& D, int /*slab_stride*/) {
  return (mlp_lds_bytes(D) + 15) & ~(size_t)15;
}
// a launch walking fpw fine slabs keeps the per-CU workgroup count of the one-slab launch (two
// for the one-tile-per-slice kernel at DLAP_BWD1_WPS = 2)
bool mlp_bwd_fpw_fits(const MlpDims& D, int KS1, int slab_stride, int tps, int fpw) {
  if (fpw > 1 && !D.wide && !(KS1 == 2 && tps == 1)) return false;     // not instantiated
  const size_t per_cu = 160 * 1024 / (tps == 1 ? DLAP_BWD1_WPS : 1);
  return mlp_bwd_lds_bytes(D, slab_stride, fpw) <= per_cu;
}
size_t mlp_bwd_lds_bytes(const MlpDims& D, int slab_stride, int fpw) {
  const size_t a = mlp_lds_bytes(D), b = (size_t)slab_stride * 4;
  return fpw > 1 ? bwd_red_off(D, slab_stride) + 2 * b : (a > b ? a : b);
}

template <class P>
static bool launch_mlp_fwd_p(const MlpJob* jobs, dim3 grid, dim3 block, size_t sh, const MlpDims& D, int KS1,
                             int WMB, hipStream_t st, bool so) {
  if (so && !P::kF32) {      // (SDF-only: the moment width is irrelevant)
    if (KS1 == 2) { hipLaunchKernelGGL((k_mlp_fwd<P, 2, 1, false, true>), grid, block, sh, st, jobs, D); HIP_OK(hipGetLastError()); return true; }
    if (KS1 == 4) { hipLaunchKernelGGL((k_mlp_fwd<P, 4, 1, false, true>), grid, block, sh, st, jobs, D); HIP_OK(hipGetLastError()); return true; }
  }
#define F_CASE(K, W) if (KS1 == K && WMB == W) { hipLaunchKernelGGL((k_mlp_fwd<P, K, W, false>), grid, block, sh, st, jobs, D); HIP_OK(hipGetLastError()); return true; }
  F_CASE(2, 1) F_CASE(2, 2) F_CASE(2, 4) F_CASE(4, 1) F_CASE(4, 2) F_CASE(4, 4)
#undef F_CASE
  return false;
}

void launch_mlp_fwd(const MlpJob* jobs, int njobs, int gx, const MlpDims& D, int KS1, int WMB,
                    hipStream_t st, bool so) {
  dim3 grid(gx, njobs), block(256);
  size_t sh = mlp_lds_bytes(D);
  if (D.wide) {      // layer 0 from k_proj0's z (bf16, or fp32 reference precision)
#define FZ_CASE(PR, W) if (WMB == W) { hipLaunchKernelGGL((k_mlp_fwd<PR, 2, W, true>), grid, block, sh, st, jobs, D); HIP_OK(hipGetLastError()); return; }
    if (D.fp32) { FZ_CASE(PrecF32, 1) FZ_CASE(PrecF32, 2) FZ_CASE(PrecF32, 4) }
    else { FZ_CASE(PrecBF16, 1) FZ_CASE(PrecBF16, 2) FZ_CASE(PrecBF16, 4) }
#undef FZ_CASE
  }
  const bool ok = D.fp32 ? launch_mlp_fwd_p<PrecF32>(jobs, grid, block, sh, D, KS1, WMB, st, so)
                         : launch_mlp_fwd_p<PrecBF16>(jobs, grid, block, sh, D, KS1, WMB, st, so);
  if (!ok) dlap_throw_hip(hipErrorInvalidValue, "mlp_fwd: unsupported (KS1, WMB)", __FILE__, __LINE__);
}

// Fused LSTM + training tower forward (k_mlp_fwd_rnn): grid (1 + gx, jobs). Instantiated for
// the paper / sweep LSTM widths (H = 4: DPP gate gathers, H = 8) on the fused layer-0 path;
// returns false for anything else (the caller then launches the LSTM and the towers separately).
static size_t fwd_rnn_lds(const MlpDims& D0, int H, int tmax) {
  MlpDims D = D0;
  D.pp_lds_floats = 0;
  return std::max(lds_bytes_of(D), gls_lds_floats_ready(tmax, H) * sizeof(float));
}
bool mlp_fwd_rnn_supported(const MlpDims& D, int KS1, int WMB, int H, int nrnn, int tmax) {
  if (D.wide || nrnn <= 0 || D.Dm != H || tmax <= 0) return false;
  if (!(H == 4 || (H == 8 && !D.fp32))) return false;
  if (!(KS1 == 2 || KS1 == 4) || !(WMB == 1 || WMB == 2 || WMB == 4)) return false;
  return fwd_rnn_lds(D, H, tmax) <= 64 * 1024;
}
// Workgroups of the fused kernel the whole device holds at once (occupancy query x CUs): the
// engine launches it only with (1 + gx) * njobs at most this, so every tower workgroup is
// co-resident with the LSTM workgroup it waits for -- forward progress does not rest on the
// dispatch order. 0 = not instantiated for this shape.
int mlp_fwd_rnn_capacity(const MlpDims& D0, int KS1, int WMB, int H, int nrnn, int tmax) {
  if (!mlp_fwd_rnn_supported(D0, KS1, WMB, H, nrnn, tmax)) return 0;
  const size_t sh = fwd_rnn_lds(D0, H, tmax);
  int per_cu = 0;
#define O_CASE(PR, K, W, HM, DP) \
  if (KS1 == K && WMB == W && H == HM) \
    HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_mlp_fwd_rnn<PR, K, W, HM, DP>, 256, sh));
#define O_KW(PR, HM, DP) O_CASE(PR, 2, 1, HM, DP) O_CASE(PR, 2, 2, HM, DP) O_CASE(PR, 2, 4, HM, DP) \
  O_CASE(PR, 4, 1, HM, DP) O_CASE(PR, 4, 2, HM, DP) O_CASE(PR, 4, 4, HM, DP)
  if (D0.fp32) { O_KW(PrecF32, 4, true) }
  else { O_KW(PrecBF16, 4, true) O_KW(PrecBF16, 8, false) }
#undef O_KW
#undef O_CASE
  // the SDF-only instantiation (launch_mlp_fwd_rnn, so = true: the phase-1/3 training and
  // evaluation forwards) has its own register footprint: the capacity is the smaller of the two
  if (!D0.fp32 && per_cu > 0) {
    int per_so = per_cu;
#define OS_CASE(K, HM, DP) \
    if (KS1 == K && H == HM) \
      HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_so, k_mlp_fwd_rnn<PrecBF16, K, 1, HM, DP, true>, 256, sh));
    OS_CASE(2, 4, true) OS_CASE(4, 4, true) OS_CASE(2, 8, false) OS_CASE(4, 8, false)
#undef OS_CASE
    per_cu = std::min(per_cu, per_so);
  }
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  int ncu = 0;
  HIP_OK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  return per_cu * ncu;
}

bool launch_mlp_fwd_rnn(const MlpJob* jobs, const RnnJob* rjobs, const ModelDesc* md, int njobs, int gx,
                        const MlpDims& D0, int KS1, int WMB, int H, int nrnn, int tmax, hipStream_t st, bool so,
                        int ne, bool selfproj, int* esig) {
  if (!mlp_fwd_rnn_supported(D0, KS1, WMB, H, nrnn, tmax))
    dlap_throw_hip(hipErrorInvalidValue, "mlp_fwd_rnn: unsupported shape", __FILE__, __LINE__);
  MlpDims D = D0;
  D.pp_lds_floats = 0;                 // the per-period inputs are read as they are published
  const size_t sh = fwd_rnn_lds(D0, H, tmax);
  dim3 grid(gx + 1 + ne, njobs), block(256);
  if (so && !D.fp32) {
#define RS_CASE(K, HM, DP) \
    if (KS1 == K && H == HM) { \
      hipLaunchKernelGGL((k_mlp_fwd_rnn<PrecBF16, K, 1, HM, DP, true>), grid, block, sh, st, jobs, D, rjobs, md, ne, (int)selfproj, esig); \
      HIP_OK(hipGetLastError()); return true; }
    RS_CASE(2, 4, true) RS_CASE(4, 4, true) RS_CASE(2, 8, false) RS_CASE(4, 8, false)
#undef RS_CASE
  }
#define R_CASE(PR, K, W, HM, DP) \
  if (KS1 == K && WMB == W && H == HM) { \
    hipLaunchKernelGGL((k_mlp_fwd_rnn<PR, K, W, HM, DP>), grid, block, sh, st, jobs, D, rjobs, md, ne, (int)selfproj, esig); \
    HIP_OK(hipGetLastError()); return true; }
#define R_KW(PR, HM, DP) R_CASE(PR, 2, 1, HM, DP) R_CASE(PR, 2, 2, HM, DP) R_CASE(PR, 2, 4, HM, DP) \
  R_CASE(PR, 4, 1, HM, DP) R_CASE(PR, 4, 2, HM, DP) R_CASE(PR, 4, 4, HM, DP)
  if (D.fp32) { R_KW(PrecF32, 4, true) }
  else { R_KW(PrecBF16, 4, true) R_KW(PrecBF16, 8, false) }
#undef R_KW
#undef R_CASE
  dlap_throw_hip(hipErrorInvalidValue, "mlp_fwd_rnn: no instantiation", __FILE__, __LINE__);
  return false;
}

void launch_mlp_fwd_zx(const MlpJob* jobs, int njobs, int gx, const MlpDims& D, int WMB, hipStream_t st,
                       bool train) {
  dim3 grid(gx, njobs), block(512);
  const size_t sh = ((lds_bytes_of(D) + 15) & ~(size_t)15) + (size_t)(4 + WMB) * D.KSX * 1024;
#define ZX_CASE(W, TR) if (WMB == W && train == TR) { hipLaunchKernelGGL((k_mlp_fwd_zx<W, TR>), grid, block, sh, st, jobs, D); HIP_OK(hipGetLastError()); return; }
  ZX_CASE(1, false) ZX_CASE(2, false) ZX_CASE(4, false) ZX_CASE(1, true) ZX_CASE(2, true) ZX_CASE(4, true)
#undef ZX_CASE
  dlap_throw_hip(hipErrorInvalidValue, "mlp_fwd_zx: unsupported moment width", __FILE__, __LINE__);
}

template <class P>
static bool launch_bwd_sdf_p(const MlpJob* jobs, dim3 grid, dim3 block, size_t sh, int tps, const MlpDims& D,
                             int KS1, int slab_stride, int roff, int fpw, hipStream_t st) {
#define S_CASE(K, N, T) if (fpw == 1 && KS1 == K && D.nl_sdf == N && tps == T) { hipLaunchKernelGGL((k_mlp_bwd_sdf<P, K, N, T, false, 1>), grid, block, sh, st, jobs, D, slab_stride, roff); HIP_OK(hipGetLastError()); return true; }
  S_CASE(2, 1, 1) S_CASE(2, 2, 1) S_CASE(2, 3, 1) S_CASE(2, 4, 1)
  S_CASE(2, 2, 2)
  S_CASE(4, 1, 1) S_CASE(4, 2, 1) S_CASE(4, 3, 1) S_CASE(4, 4, 1)
#undef S_CASE
  // several fine slabs per workgroup (batched models): the one-tile-per-slice tower of the
  // 64-column X (mlp_bwd_fpw_supported)
#define SF_CASE(N) if (fpw > 1 && KS1 == 2 && D.nl_sdf == N && tps == 1) { hipLaunchKernelGGL((k_mlp_bwd_sdf<P, 2, N, 1, false, 0>), grid, block, sh, st, jobs, D, slab_stride, roff); HIP_OK(hipGetLastError()); return true; }
  SF_CASE(1) SF_CASE(2) SF_CASE(3) SF_CASE(4)
#undef SF_CASE
  return false;
}

void launch_mlp_bwd_sdf(const MlpJob* jobs, int njobs, int gx, int nslice, int tps, const MlpDims& D,
                        int KS1, int slab_stride, int fpw, hipStream_t st) {
  dim3 grid(gx, njobs, nslice), block(256);
  const size_t sh = mlp_bwd_lds_bytes(D, slab_stride, fpw);
  const int roff = fpw > 1 ? (int)bwd_red_off(D, slab_stride) : 0;
  if (D.wide) {
#define SZ_CASE(PR, N, T) if (D.nl_sdf == N && tps == T) { hipLaunchKernelGGL((k_mlp_bwd_sdf<PR, 2, N, T, true, 0>), grid, block, sh, st, jobs, D, slab_stride, roff); HIP_OK(hipGetLastError()); return; }
    if (D.fp32) { SZ_CASE(PrecF32, 1, 1) SZ_CASE(PrecF32, 2, 1) SZ_CASE(PrecF32, 3, 1) SZ_CASE(PrecF32, 4, 1) SZ_CASE(PrecF32, 2, 2) }
    else { SZ_CASE(PrecBF16, 1, 1) SZ_CASE(PrecBF16, 2, 1) SZ_CASE(PrecBF16, 3, 1) SZ_CASE(PrecBF16, 4, 1) SZ_CASE(PrecBF16, 2, 2) }
#undef SZ_CASE
    dlap_throw_hip(hipErrorInvalidValue, "mlp_bwd_sdf: unsupported depth (wide)", __FILE__, __LINE__);
  }
  const bool ok = D.fp32 ? launch_bwd_sdf_p<PrecF32>(jobs, grid, block, sh, tps, D, KS1, slab_stride, roff, fpw, st)
                         : launch_bwd_sdf_p<PrecBF16>(jobs, grid, block, sh, tps, D, KS1, slab_stride, roff, fpw, st);
  if (!ok) dlap_throw_hip(hipErrorInvalidValue, "mlp_bwd_sdf: unsupported depth/tiling", __FILE__, __LINE__);
}

template <class P>
static bool launch_bwd_mom_p(const MlpJob* jobs, dim3 grid, dim3 block, size_t sh, int tps, const MlpDims& D,
                             int KS1, int WMB, int slab_stride, int roff, hipStream_t st) {
#define M_CASE(K, W, N) if (KS1 == K && WMB == W && D.nl_mom == N && tps == 1) { hipLaunchKernelGGL((k_mlp_bwd_mom<P, K, W, N, 1, false>), grid, block, sh, st, jobs, D, slab_stride, roff); HIP_OK(hipGetLastError()); return true; }
  M_CASE(2, 1, 1) M_CASE(2, 2, 1) M_CASE(2, 4, 1)
  M_CASE(2, 1, 2) M_CASE(2, 2, 2) M_CASE(2, 4, 2)
  M_CASE(2, 1, 3) M_CASE(2, 2, 3) M_CASE(2, 4, 3)
  M_CASE(4, 1, 1) M_CASE(4, 2, 1) M_CASE(4, 4, 1)
  M_CASE(4, 1, 2) M_CASE(4, 2, 2) M_CASE(4, 4, 2)
#undef M_CASE
  return false;
}

void launch_mlp_bwd_mom(const MlpJob* jobs, int njobs, int gx, int nslice, int tps, const MlpDims& D,
                        int KS1, int WMB, int slab_stride, int fpw, hipStream_t st) {
  dim3 grid(gx, njobs, nslice), block(256);
  const size_t sh = mlp_bwd_lds_bytes(D, slab_stride, fpw);
  const int roff = fpw > 1 ? (int)bwd_red_off(D, slab_stride) : 0;
  if (D.wide) {
#define MZ_CASE(PR, W, N) if (WMB == W && D.nl_mom == N && tps == 1) { hipLaunchKernelGGL((k_mlp_bwd_mom<PR, 2, W, N, 1, true>), grid, block, sh, st, jobs, D, slab_stride, roff); HIP_OK(hipGetLastError()); return; }
    if (D.fp32) {
      MZ_CASE(PrecF32, 1, 1) MZ_CASE(PrecF32, 2, 1) MZ_CASE(PrecF32, 4, 1)
      MZ_CASE(PrecF32, 1, 2) MZ_CASE(PrecF32, 2, 2) MZ_CASE(PrecF32, 4, 2)
      MZ_CASE(PrecF32, 1, 3) MZ_CASE(PrecF32, 2, 3) MZ_CASE(PrecF32, 4, 3)
    } else {
      MZ_CASE(PrecBF16, 1, 1) MZ_CASE(PrecBF16, 2, 1) MZ_CASE(PrecBF16, 4, 1)
      MZ_CASE(PrecBF16, 1, 2) MZ_CASE(PrecBF16, 2, 2) MZ_CASE(PrecBF16, 4, 2)
      MZ_CASE(PrecBF16, 1, 3) MZ_CASE(PrecBF16, 2, 3) MZ_CASE(PrecBF16, 4, 3)
    }
#undef MZ_CASE
    dlap_throw_hip(hipErrorInvalidValue, "mlp_bwd_mom: unsupported depth/width (wide)", __FILE__, __LINE__);
  }
  const bool ok = D.fp32 ? launch_bwd_mom_p<PrecF32>(jobs, grid, block, sh, tps, D, KS1, WMB, slab_stride, roff, st)
                         : launch_bwd_mom_p<PrecBF16>(jobs, grid, block, sh, tps, D, KS1, WMB, slab_stride, roff, st);
  if (!ok) dlap_throw_hip(hipErrorInvalidValue, "mlp_bwd_mom: unsupported depth/width", __FILE__, __LINE__);
}

std::vector<long long> mlp_timestamps() {
  std::vector<long long> v(24);
  HIP_OK(hipMemcpyFromSymbol(v.data(), HIP_SYMBOL(g_mlp_ts), sizeof(long long) * 24));
  return v;
}
