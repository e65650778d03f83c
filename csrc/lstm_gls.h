// The gate-per-lane LSTM recurrence with every per-step output kept in LDS (k_lstm_gls), shared
// by the stand-alone prologue kernel (k_rnn.hip) and the fused LSTM + training-tower forward
// (k_mlp_fwd_rnn in k_mlp.hip), where it runs on wave 0 of workgroup 0 and publishes its
// progress period by period to the tower workgroups.
//
// Reference: `MacroLSTM.forward` (`/root/reference/src/model.py:21-84`), one nn.LSTM over the
// T-sequence with batch 1, PyTorch gate order i, f, g, o, both biases.
#pragma once
#include "common.h"
#include "layout.h"
#include "rnn.h"

// sum_j w[j] * v(lane j) as a balanced tree (dependency depth log2 HM + 1)
template <int HM>
DLAP_DEV float bcast_dot(const float (&w)[HM], float v) {
#pragma clang fp contract(off)
  float p[HM];
#pragma unroll
  for (int j = 0; j < HM; ++j) p[j] = w[j] * __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
#pragma unroll
  for (int w2 = 1; w2 < HM; w2 *= 2)
#pragma unroll
    for (int j = 0; j + w2 < HM; j += 2 * w2) p[j] += p[j + w2];
  return p[0];
}

// Same dot product with h_j taken from lane j of the lane's own 16-lane row by a DPP
// row_newbcast operand (gfx90a+): no VALU -> SGPR -> VALU round trip through v_readlane on the
// recurrence's critical path. Valid when every lane that uses the result sits in row 0 and the
// source units are lanes 0..HM-1 (the gate-per-lane form with 4H <= 16).
template <int J>
DLAP_DEV float row_bcast(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x150 + J, 0xF, 0xF, true));
}
// acc + sum_j w[j] h_j: the accumulator (the step's input projection) enters the first FMA, so the
// chain is FMA | FMA | add (three dependent levels) instead of mul | fma | add | add
template <int HM>
DLAP_DEV float bcast_dot_row(const float (&w)[HM], float v, float acc = 0.f) {
  static_assert(HM >= 1 && HM <= 4, "row-broadcast dot: 1..4 units");
  float p0 = fmaf(w[0], row_bcast<0>(v), acc);
  if constexpr (HM == 1) return p0;
  float p1 = w[1] * row_bcast<1>(v);
  if constexpr (HM == 2) return p0 + p1;
  p0 = fmaf(w[2], row_bcast<2>(v), p0);
  if constexpr (HM == 3) return p0 + p1;
  p1 = fmaf(w[3], row_bcast<3>(v), p1);
  return p0 + p1;
}

// Gate-per-lane gather: lane L owns gate row L (q = L / H, unit L % H); the f/g/o values are
// moved onto the unit lanes (DPP row rotates when 4H <= 16, ds_bpermute otherwise).
template <int HM, bool DPPG>
DLAP_DEV float gl_gather(float y, int off_units, int q) {
  if constexpr (DPPG) {
    // lane l receives lane (l - n) mod 16 for row_ror:n  ->  n = 16 - q*H reads lane l + q*H
    if (q == 1) return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(y), 0x120 + (16 - HM), 0xF, 0xF, false));
    if (q == 2) return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(y), 0x120 + (16 - 2 * HM), 0xF, 0xF, false));
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(y), 0x120 + (16 - 3 * HM), 0xF, 0xF, false));
  } else {
    return __shfl(y, (int)(threadIdx.x & 63) + off_units, 64);
  }
}

// ---- layer-0 input projection (k_proj in k_rnn.hip, and the fused forward's in-kernel form) ----
// xg[t] = W_ih x_t + b_ih + b_hh (layer-0 LSTM gates) and abias[t] = W_m0[:, :M] x_t + b_m0
// (moment layer-0 per-period bias, zero-padded to 64): a [T x MP] . [MP x NP] fp32 GEMM on
// the matrix cores. grid (ceil(T/16), NP/16, jobs), one wave per 16x16 output tile, K = 4 per
// v_mfma_f32_16x16x4f32 (full fp32 products / accumulation). Operands come straight from
// global memory (macro rows, and the k_pack-produced wproj [MP+2][NP] whose last two rows
// hold the biases): all loads of a tile are independent, so the tile costs ~one memory round trip.
//   A (16x4): lane l -> A[t = l&15][k = l>>4];  B (4x16): lane l -> B[k = l>>4][o = l&15]
//   C (16x16): lane l -> C[t = 4*(l>>4) + r][o = l&15]
// One 16 (periods) x 16 (outputs) tile of the projection on one wave: returns lane l's
// accumulator C[t0 + 4*(l>>4) + r][o0 + (l&15)] with the bias added.
// Operands through raw buffer loads: one 32-bit per-lane offset per operand stream with the
// K step in the instruction's immediate (x) or a scalar offset (w), so a chunk's 2 x PROJ_KC
// loads cost their data registers only and stay in flight together even inside a kernel at its
// register limit (the fused forward's in-kernel projection; with 64-bit per-load addresses the
// compiler there serialised them, one memory round trip per load). Reads past a row end are
// masked to zero; reads past the buffer return zero (the descriptors' num_records).
DLAP_DEV f32x4 proj_tile(const RnnJob& J, const ModelDesc* md, int t0, int o0) {
  const int T = J.T, M = md->M, MP = md->proj_mp, NP = md->proj_np;
  const int l = threadIdx.x & 63, n = l & 15, kq = l >> 4;
  const int ta = min(t0 + n, T - 1);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)J.macro, (short)0, T * M * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)J.wproj, (short)0, (MP + 2) * NP * 4, 0x00020000);
  const int xo = (ta * M + kq) * 4, wo = (kq * NP + o0 + n) * 4;
  f32x4 acc = zero4();
  // all operand loads of a K chunk are issued before the first MFMA consumes them: one
  // memory round trip per PROJ_KC * 4 columns instead of one per unrolled group
  constexpr int PROJ_KC = 48;
  for (int kb = 0; kb < MP; kb += 4 * PROJ_KC) {
    float a[PROJ_KC], b[PROJ_KC];
#pragma unroll
    for (int s = 0; s < PROJ_KC; ++s) {
      a[s] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, xo + 4 * kb + 16 * s, 0, 0));
      b[s] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(wr, wo, (kb + 4 * s) * NP * 4, 0));
    }
#pragma unroll
    for (int s = 0; s < PROJ_KC; ++s) {
      const int m = kb + 4 * s + kq;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(m < M ? a[s] : 0.f, m < MP ? b[s] : 0.f, acc, 0, 0, 0);
    }
  }
  const auto wcol = gp(J.wproj) + o0 + n;
  const float bias = wcol[(size_t)MP * NP] + wcol[(size_t)(MP + 1) * NP];   // b_ih + b_hh (b_m0 + 0)
  return acc + bias;
}


// The fused forward's in-kernel projection (k_mlp_fwd_rnn, selfproj): waves w0 .. w0 + nw - 1 of
// the recurrence's workgroup take the 16-period tiles of xg round-robin -- proj_tile, the bits of
// k_proj -- write them to the LDS staging area and raise each tile's ready flag once the wave's
// LDS stores have completed; the recurrence (lstm_gls_body, `ready`) polls a tile's flag (plain
// LDS reads: no fence -- a wave's LDS operations complete in order) only when it reaches a tile
// it has not seen ready yet.
// Fast path (one 16-wide gate tile, MP <= 192: the common LSTM[4]): the weight column fragment is
// loaded once per wave and the next tile's macro rows are in flight while the MFMAs of the
// current one run (ping-pong register sets; the fused forward is at its register limit anyway,
// so the extra set is free) -- a tile every ~memory round trip per wave instead of a round trip
// plus the MFMA chain; the same operands and MFMA order as proj_tile.
DLAP_DEV void proj_into_lds(const RnnJob& J, const ModelDesc* __restrict__ md, float* sx, int* ready, int w, int nw,
                            long long* ts = nullptr) {
  const int T = J.T, G4 = 4 * md->H;
  const int l = threadIdx.x & 63, n = l & 15, kq = l >> 4;
  constexpr int KC = 48;
  const int M = md->M, MP = md->proj_mp, NP = md->proj_np;
  if (G4 == 16 && MP <= 4 * KC) {
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)J.macro, (short)0, T * M * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)J.wproj, (short)0, (MP + 2) * NP * 4, 0x00020000);
    float b[KC], a0[KC], a1[KC];
    const int wo = (kq * NP + n) * 4;
#pragma unroll
    for (int s = 0; s < KC; ++s) b[s] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(wr, wo, 4 * s * NP * 4, 0));
    const auto wcol = gp(J.wproj) + n;
    const float bias = wcol[(size_t)MP * NP] + wcol[(size_t)(MP + 1) * NP];
    auto load_a = [&](int j, float (&a)[KC]) {
      const int ta = min(16 * j + n, T - 1);
      const int xo = (ta * M + kq) * 4;
#pragma unroll
      for (int s = 0; s < KC; ++s) a[s] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, xo + 16 * s, 0, 0));
    };
    auto tile = [&](int j, const float (&a)[KC]) {
      f32x4 acc = zero4();
#pragma unroll
      for (int s = 0; s < KC; ++s) {
        const int m = 4 * s + kq;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(m < M ? a[s] : 0.f, m < MP ? b[s] : 0.f, acc, 0, 0, 0);
      }
      acc = acc + bias;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * j + 4 * kq + r;
        if (t < T) sx[t * G4 + n] = acc[r];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (l == 0) __hip_atomic_store(ready + j, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (ts && l == 0 && j == w) ts[0] = wall_clock64();               // (timing: first tile done)
    };
    if (ts && l == 0) ts[1] = wall_clock64();                           // (timing: weights requested)
    int j = w;
    if (j * 16 < T) load_a(j, a0);
    while (j * 16 < T) {
      if ((j + nw) * 16 < T) load_a(j + nw, a1);
      tile(j, a0);
      j += nw;
      if (j * 16 >= T) break;
      if ((j + nw) * 16 < T) load_a(j + nw, a0);
      tile(j, a1);
      j += nw;
    }
    return;
  }
  for (int j = w; j * 16 < T; j += nw) {
    for (int o0 = 0; o0 < G4; o0 += 16) {
      const f32x4 acc = proj_tile(J, md, 16 * j, o0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * j + 4 * kq + r;
        if (t < T && o0 + n < G4) sx[t * G4 + o0 + n] = acc[r];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (l == 0) __hip_atomic_store(ready + j, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}
// the recurrence waits for the projected tile holding period t (one wave; bounded). `have`:
// tiles 0 .. have - 1 are known to be ready (the recurrence reaches the tiles in order)
DLAP_DEV void wait_xtile(const int* ready, int t, int& have) {
  if (!ready || (t >> 4) < have) return;
  const int j = t >> 4;
  unsigned spins = 0;
  while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(ready + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) == 0) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1u << 24)) break;         // (never: the producing waves always finish)
  }
  asm volatile("" ::: "memory");
  have = j + 1;
}

// LDS ordering among the lanes of ONE wave (the recurrence runs on a single wave; the fused
// kernel's publisher wave never takes part in a workgroup barrier, so none is used here).
DLAP_DEV void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// LDS (floats): xg [T][4H] | gates [T][4H] | cells [T][H] | outputs 2 x [T][H] | junk [64].
__host__ __device__ inline size_t gls_lds_floats(int T, int H) { return (size_t)T * (8 * H + 3 * H) + 64; }
// ready flags after the recurrence's LDS image (one per 16-period tile)
__host__ __device__ inline size_t gls_ready_offset(int T, int H) { return gls_lds_floats(T, H); }
__host__ __device__ inline size_t gls_lds_floats_ready(int T, int H) { return gls_lds_floats(T, H) + (T + 15) / 16 + 4; }
// the last layer's output ring inside that image
__host__ __device__ inline size_t gls_out_offset(int T, int H, int nrnn) {
  return (size_t)T * (8 * H + H) + (size_t)((nrnn - 1) & 1) * T * H;
}

// The recurrence on one wave (lanes = threadIdx.x & 63). The serial loop is branch-free (all 64
// lanes run the same instructions, results on non-owner lanes are discarded with selects and go
// to a junk slot) and issues three ds_write per step. The saved gates / cells / outputs are
// flushed to global memory once per layer with coalesced stores; a deeper layer reads its input
// from the LDS ring directly. Tanh of the g gate and of the cell use 2 sigm(2x) - 1 (absolute
// error ~1e-7, fp32 rounding level for the cell update).
//   STAGEX: copy the layer-0 input projections xg (global) into LDS first (else the caller
//           has put them there);
//   PUB:    every 8 steps of the last layer store the number of finished periods to *sprog
//           (LDS, workgroup-scope release); the output flush to J.out is left to the
//           publisher wave (lstm_publish in k_mlp.hip).
//   ts:     optional in-kernel timestamps (slots tsb + 1, tsb + 2, tsb + 3).
//   ready:  (fused forward, in-kernel projection) per-tile flags of the staged projections: the
//           layer-0 loop waits for a tile before it reads its steps (nullptr: all staged).
template <int HM, bool DPPG, bool STAGEX, bool PUB>
DLAP_DEV void lstm_gls_body(const RnnJob& J, const ModelDesc* __restrict__ md, float* sm, int* sprog,
                            long long* ts, int tsb, const int* ready = nullptr) {
  // every multiply-add of the recurrence is written out (fmaf) and nothing else is contracted: the
  // stand-alone kernel and the fused forward compile this body in different contexts and must
  // produce the same bits (tests/test_invariance_gpu.py, fused vs two launches)
#pragma clang fp contract(off)
  const int nrnn = md->nrnn;
  const int T = J.T, H = DPPG ? HM : md->H, G4 = 4 * H;
  const int L = threadIdx.x & 63;
  auto stamp = [&](int slot) { if (ts && L == 0) ts[tsb + slot] = wall_clock64(); };
  auto publish = [&](int v) {
    if constexpr (PUB) __hip_atomic_store(sprog, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  // the recurrence is one latency-bound wave: top issue priority on its SIMD, so the tower waves
  // of a concurrent branch (pipelined evaluation / training) do not stretch its serial chain
  __builtin_amdgcn_s_setprio(3);
  const bool gl = L < G4, ul = L < H;
  const int row = gl ? L : 0;
  const bool is_g = gl && L >= 2 * H && L < 3 * H;
  // Pre-scaled exponent domain: a gate row's pre-activation is carried as kx * pre with
  // kx = -ka log2(e), so act = kb / (1 + exp2(.)) + kc needs no multiply on the chain. The
  // cell is carried as c' = KC c (KC = -2 log2 e), so tanh(c) = 2 / (1 + exp2(c')) - 1; the
  // g lanes produce KC g directly (kb, kc scaled by KC) so c' = f c' + i (KC g).
  constexpr float LOG2E = 1.4426950408889634f;
  constexpr float KC = -2.f * LOG2E;
  const float kx = is_g ? -2.f * LOG2E : -LOG2E;
  const float kb = is_g ? 2.f * KC : 1.f, kc = is_g ? -KC : 0.f;
  const float ysave = is_g ? 1.f / KC : 1.f;      // saved gates are the unscaled activations
  const bool drop = J.train && J.dropout > 0.f;
  const uint32_t thr = (uint32_t)(J.dropout * 16777216.f + 0.5f);
  const float scale = drop ? 1.f / (1.f - J.dropout) : 1.f;
  const uint32_t step = J.step ? (uint32_t)*gp(J.step) : 0u;
  const auto params = gp(J.params);
  const bool save = J.sc != nullptr;
  float* sx = sm;
  float* sgb = sx + (size_t)T * G4;
  float* scb = sgb + (size_t)T * G4;
  float* shb0 = scb + (size_t)T * H;
  float* junk = shb0 + (size_t)2 * T * H;
  if constexpr (STAGEX) {
    const auto xg = gp(J.xg);
    for (int i = L; i < T * G4; i += 64) sx[i] = xg[i];
    wave_lds_sync();
  }
  for (int l = 0; l < nrnn; ++l) {
    const bool last = l + 1 == nrnn;
    float whh[HM], wih[HM];
#pragma unroll
    for (int j = 0; j < HM; ++j) {
      const bool ok = gl && j < H;
      const int jj = j < H ? j : 0;
      const float a = params[md->lstm_w_hh[l] + row * H + jj];
      const float b = l > 0 ? params[md->lstm_w_ih[l] + row * H + jj] : 0.f;
      whh[j] = ok ? a * kx : 0.f;
      wih[j] = ok ? b * kx : 0.f;
    }
    const float bb = l > 0 ? params[md->lstm_b_ih[l] + row] + params[md->lstm_b_hh[l] + row] : 0.f;
    const float bias = gl ? bb * kx : 0.f;
    if (l == 0) stamp(1);
    float* shb = shb0 + (size_t)(l & 1) * T * H;            // this layer's outputs
    const float* sin = shb0 + (size_t)((l + 1) & 1) * T * H; // previous layer's outputs
    // per-lane LDS destinations (non-owner lanes write their junk slot)
    float* gdst = gl ? sgb + L : junk + L;
    float* udst_c = ul ? scb + L : junk + L;
    float* udst_h = ul ? shb + L : junk + L;
    const int gstride = gl ? G4 : 0, ustride = ul ? H : 0;
    // h / c on lanes >= H are bounded garbage: the broadcast reads lanes j < HM only, and
    // lanes H <= j < HM carry zero weights
    float h = ul && J.h0 ? gp(J.h0)[l * H + L] : 0.f, c = ul && J.c0 ? gp(J.c0)[l * H + L] * KC : 0.f;
    auto cell = [&](int t, float pre) {
      if constexpr (DPPG) pre = bcast_dot_row<HM>(whh, h, pre);
      else pre += bcast_dot<HM>(whh, h);
      const float y = fmaf(kb, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(pre)), kc);
      const float gf = gl_gather<HM, DPPG>(y, H, 1);
      const float gg = gl_gather<HM, DPPG>(y, 2 * H, 2);
      const float go = gl_gather<HM, DPPG>(y, 3 * H, 3);
      c = fmaf(gf, c, y * gg);                              // y = i on the unit lanes
      h = go * fmaf(2.f, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(c)), -1.f);
      gdst[t * gstride] = y * ysave;
      udst_c[t * ustride] = c * (1.f / KC);
      udst_h[t * ustride] = h;
    };
    if (l == 0) {
      // inputs in chunks of CH steps, the next chunk's LDS reads issued a whole chunk ahead:
      // inside a chunk the recurrence has no LDS load (and no wait on the per-step LDS stores,
      // which a one-step-ahead read kept on the chain through the shared LDS counter)
      constexpr int CH = 8;
      float xa[CH], xb[CH];
      auto ldch = [&](int t0, float (&x)[CH]) {
#pragma unroll
        for (int k = 0; k < CH; ++k) x[k] = sx[min(t0 + k, T - 1) * G4 + row];
      };
      const int tfull = T / CH * CH;
      int have = 0;                                     // projected tiles known to be in LDS
      wait_xtile(ready, 0, have);
      ldch(0, xa);
      for (int t0 = 0; t0 < tfull; t0 += CH) {
        if (t0 + CH < T) wait_xtile(ready, t0 + CH, have);   // (CH divides 16: one tile per chunk)
        ldch(t0 + CH, xb);
#pragma unroll
        for (int k = 0; k < CH; ++k) cell(t0 + k, xa[k] * kx);
#pragma unroll
        for (int k = 0; k < CH; ++k) xa[k] = xb[k];
        if (PUB && last) publish(t0 + CH);
      }
      for (int t = tfull; t < T; ++t) {
        wait_xtile(ready, t, have);
        cell(t, sx[t * G4 + row] * kx);
      }
    } else {
      const uint32_t key_in = dropout_key(J.seed, step, 32 + (l - 1));
      float nx = ul ? sin[L] : 0.f;
      for (int t = 0; t < T; ++t) {
        float xv = ul ? nx : 0.f;
        nx = sin[(t + 1 < T ? t + 1 : t) * H + (ul ? L : 0)];
        if (drop) xv = dropout_keep(key_in, (uint32_t)t, (uint32_t)(ul ? L : 0), thr) ? xv * scale : 0.f;
        float pre = bias;
#pragma unroll
        for (int j = 0; j < HM; ++j)
          pre = fmaf(wih[j], __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xv), j)), pre);
        cell(t, pre);
        if (PUB && last && (t & 7) == 7) publish(t + 1);
      }
    }
    if (PUB && last) publish(T);
    if (l == 0) stamp(2);
    wave_lds_sync();
    // flush: saved gates / cells / outputs (train), tower input (last layer)
    if (save) {
      const auto sg = gp(J.sg) + (size_t)l * T * G4;
      const auto sc = gp(J.sc) + (size_t)l * T * H;
      const auto sh = gp(J.sh) + (size_t)l * T * H;
      for (int i = L; i < T * G4; i += 64) sg[i] = sgb[i];
      for (int i = L; i < T * H; i += 64) { sc[i] = scb[i]; sh[i] = shb[i]; }
    }
    if (last && !PUB) {
      const auto out = gp(J.out);
      for (int i = L; i < T * H; i += 64) out[i] = shb[i];
    }
    wave_lds_sync();
  }
  stamp(3);
}
