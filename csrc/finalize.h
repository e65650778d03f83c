// Gradient finalisation blocks (k_finalize in k_update.hip; also the slab / per-period blocks of
// the fused backward tail k_lstm_tail in k_rnn.hip): sums the per-workgroup slabs of the MLP
// backward into the flat gradient vector and the per-row LSTM / moment-bias gradients into
// per-period sums. Block b of the job's block space: [0, ntile*64) weight-tile elements,
// then the extra rows, then one block per period.
#pragma once
#include "common.h"
#include "layout.h"
#include "update.h"

// signal: the fused tail -- the per-period sum is stored write-through (sc1) and, once this wave
// has drained its stores, counted on *ctr (agent scope); the LSTM block of the launch polls it.
DLAP_DEV void finalize_block(const FinJob& J, const ModelDesc* __restrict__ md, int phase, int slab_stride, int b,
                             int* ctr = nullptr) {
  const bool mom = phase == 2;
  const int ntile = mom ? md->ntile_m : md->ntile_s;
  const int tps = mom ? md->tps_m : md->tps_s;
  const int nb_tiles = ntile * 64;                    // 64 elements per block
  const int nb_extra = (SLAB_EXTRA + 63) / 64;
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // slab sums: lane = element, the 4 waves split the slabs (each sums its quarter in order,
  // 16 independent loads in flight), then a fixed-order LDS combine
  // (group 4: the stored slabs are fine slabs, summed in groups ((s0 + s1) + s2) + s3 first --
  // the coarse slabs a launch with 4 fine slabs per workgroup stores; see wg_slab_finish)
  auto slab_sum = [&](const float* src) {
    const auto s0 = gp(src);
    float acc = 0.f;
    if (J.group == 4) {
      const int nc = J.nslab >> 2;
#pragma unroll 4
      for (int k = wave; k < nc; k += 4) {
        const size_t b = (size_t)4 * k * slab_stride;
        float c = s0[b] + s0[b + slab_stride];
        c += s0[b + 2 * (size_t)slab_stride];
        c += s0[b + 3 * (size_t)slab_stride];
        acc += c;
      }
    } else {
#pragma unroll 16
      for (int k = wave; k < J.nslab; k += 4) acc += s0[(size_t)k * slab_stride];
    }
    red[wave][lane] = acc;
    __syncthreads();
    return red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
  };
  // the packed training weights of layers >= 1 and the SDF output row carry the dropout scale
  // 1/(1-p) (k_pack), so their slab sums are gradients w.r.t. the scaled weights: scale back
  const float dscale = J.dropout > 0.f ? 1.f / (1.f - J.dropout) : 1.f;
  if (b < nb_tiles) {
    const int ti = b >> 6, e = ((b & 63) << 6) + lane;
    const GradTile& G = mom ? md->tile_m[ti] : md->tile_s[ti];
    // slab position e of the tile: natural (o, i) = (e >> 6, e & 63), or (the one-pass SDF backward,
    // k_tbwd.hip) the MFMA accumulator layout -- e = ((4u + v) * 64 + 16 q + n) * 4 + r holds
    // (o, i) = (16u + 4q + r, 16v + n) -- read lane-contiguously either way
    int o = e >> 6, i = e & 63;
    if (!mom && md->tbwd) {
      const int r = e & 3, l = (e >> 2) & 63, uv = e >> 8;
      o = 16 * (uv >> 2) + 4 * (l >> 4) + r;
      i = 16 * (uv & 3) + (l & 15);
    }
    i += 64 * G.chunk;
    const int tpos = ti - G.slice * tps;
    const float v = slab_sum(J.slab + (size_t)G.slice * J.nslab * slab_stride + tpos * 4096 + e);
    bool ok = o < G.out && i < G.in;
    int col = G.col0 + i;
    if (G.xmap) {                                   // fused SDF layer 0: panel column -> W0 column
      const int F = md->F, ppc = md->md.ppc;
      if (i < F) col = i;
      else if (i >= ppc && i < ppc + md->Dm) col = F + (i - ppc);
      else ok = false;
    }
    if (wave == 0 && ok) st_wt(gp(J.grads) + G.w_off + o * G.ld + col, G.layer > 0 ? v * dscale : v);
    return;
  }
  b -= nb_tiles;
  if (b < nb_extra) {
    const int e = b * 64 + lane;
    const int ec = e < SLAB_EXTRA ? e : SLAB_EXTRA - 1;
    const float v = slab_sum(J.slab + tps * 4096 + ec);     // slice-0 slabs
    const int dst = e < SLAB_EXTRA ? (mom ? md->extra_m[e] : md->extra_s[e]) : -1;
    const bool wo = !mom && e >= DLAP_MAXL * 64 && e < DLAP_MAXL * 64 + 64;   // SDF output row
    if (wave == 0 && dst >= 0) st_wt(gp(J.grads) + dst, wo ? v * dscale : v);
    return;
  }
  b -= nb_extra;
  // per-period segment sums: one block per period, threads = (column d, row group)
  // (phase 2: only the moment layer-0 width of each [R][64] row is live -- the downstream
  // W_macro / bias gradients read dab[t][g < m[0].out] -- so only those columns are summed)
  const int D = mom ? md->m[0].out : (md->nrnn > 0 ? md->Dm : 0);
  const int t = b;
  if (D == 0 || t >= J.T) return;
  __shared__ float seg[256];
  int Dp = 1;
  while (Dp < D) Dp <<= 1;
  const int nrg = 256 / Dp, d = threadIdx.x % Dp, rg = threadIdx.x / Dp;
  const auto src = gp(mom ? J.v : J.u);
  const int ld = mom ? 64 : D;                        // row stride of v / u
  const int r0 = gp(J.row_ptr)[t], r1 = gp(J.row_ptr)[t + 1];
  if (!mom && D == 4) {
    // (the LSTM[4] per-period inputs) one 16-byte load per row: thread k sums rows r0 + k,
    // r0 + k + 256, ... in order (every load of the period issued before the first add: one
    // memory round trip for ~4k rows), then fixed xor trees per wave and the waves in order
    constexpr int RB = 16;
    const auto u4 = reinterpret_cast<const f32x4*>(&src[0]);
    f32x4 acc = zero4();
    for (int c0 = r0; c0 < r1; c0 += 256 * RB) {
      f32x4 v[RB];
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        const int r = c0 + threadIdx.x + 256 * k;
        v[k] = r < r1 ? u4[r] : zero4();
      }
#pragma unroll
      for (int k = 0; k < RB; ++k) acc = acc + v[k];
    }
    __shared__ f32x4 wred[4];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] += __shfl_xor(acc[c], o, 64);
    if ((threadIdx.x & 63) == 0) wred[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x < 4) {
      const float tot = ((wred[0][threadIdx.x] + wred[1][threadIdx.x]) + wred[2][threadIdx.x]) + wred[3][threadIdx.x];
      if (ctr) __hip_atomic_store(gp(J.dpp) + t * 4 + threadIdx.x, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else gp(J.dpp)[t * 4 + threadIdx.x] = tot;
    }
    if (ctr && threadIdx.x < 64) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  float s = 0.f;
  if (d < D) {
#pragma unroll 8
    for (int r = r0 + rg; r < r1; r += nrg) s += src[(size_t)r * ld + d];
  }
  seg[threadIdx.x] = s;
  __syncthreads();
  if (rg == 0 && d < D) {
    float tot = 0.f;
    for (int g = 0; g < nrg; ++g) tot += seg[g * Dp + d];
    if (mom && ctr) __hip_atomic_store(gp(J.dab) + t * 64 + d, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (mom) gp(J.dab)[t * 64 + d] = tot;      // (row stride 64)
    else if (ctr) __hip_atomic_store(gp(J.dpp) + t * D + d, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else gp(J.dpp)[t * D + d] = tot;
  }
  if (ctr && threadIdx.x < 64) {
    // the storing threads all sit in wave 0 (D <= 64 columns, row group 0): drain them, then one
    // agent-scope add publishes this period (R1 hand-off: write-through payload, counted signal)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
