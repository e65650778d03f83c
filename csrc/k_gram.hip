// Gram-matrix form of the moment losses while the moments are frozen (phases 1 and 3, and
// every evaluation split): SURVEY §2.3 K5/K6, VERDICT r2 "next round" item 2.
//
// Reference (`/root/reference/src/model.py:346-433`): with a_{t,i} = R_{t,i} m_{t,i} / max(T_i, 1),
//   E_{k,i} = sum_t h_{k,t,i} a_{t,i} SDF_t,   L_cond = mean_{k,i} E^2,   L_unc = the h == 1 case.
// E is linear in the SDF vector s = 1 + P, so
//   L_cond = s^T Gc s / (K N),  Gc[t][t'] = sum_{i,k} a_{t,i} a_{t',i} h_{k,t,i} h_{k,t',i},
//   L_unc  = s^T Gu s / N,      Gu[t][t'] = sum_i a_{t,i} a_{t',i},
//   dL/dSDF_t = 2 (G s)_t / (K N)  (resp. / N).
// The moments only change in phase 2, so G is built once per moment refresh (an fp64 MFMA
// GEMM over the N*K axis) and every epoch replaces the dense [K,T,N] asset passes by a T x T
// quadratic form (k_period_bwd in Gram mode, k_loss.hip). G and the quadratic form are fp64:
// the form squares the conditioning of the per-asset sums, fp32 would lose ~5 digits.
//
// k_gram_build: grid (tiles x block-slices, jobs); a workgroup = one 32x32 upper-triangle tile
// of G, its GB_WAVES waves = GB_WAVES slices of the inner axis (split-K), each as 2 x 2
// v_mfma_f64_16x16x4_f64 tiles, summed in LDS in a fixed wave order.
//   inner index e of Gc = i * K + k (h is [T][N][K], so a row of the operand is contiguous):
//   lane (r = l & 15, q = l >> 4) loads elements e0 + 4q .. +3 of row t0 + r as one 16-byte
//   load; MFMA j of the chunk takes element j (k-slot q <-> e0 + 4q + j), so the four MFMAs of
//   a 16-element chunk cover it once. Gu runs its own inner axis over stocks (4 per MFMA) in
//   both modes; unconditional-only jobs (h == nullptr) run that loop alone.
//   Block partials go to part[job][block-slice][2][T][T] (upper-triangle tiles only).
// k_gram_reduce: fixed-order sum over the slices, mirrored to the full symmetric matrices.
#include <cstdlib>
#include "common.h"
#include "loss.h"

typedef double f64x4 __attribute__((ext_vector_type(4)));

DLAP_DEV f64x4 mfma_f64(double a, double b, f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

DLAP_DEV int gram_tiles(int T) { return (T + 31) >> 5; }

#define GB_WAVES 8      // waves per workgroup: one tile, GB_WAVES inner-axis slices
#define GB_U 2          // 16-element chunks per register batch (two batches in flight)

__global__ __launch_bounds__(64 * GB_WAVES) void k_gram_build(const GramJob* __restrict__ jobs, int nsb) {
  const GramJob& J = jobs[blockIdx.y];
  const int T = J.T, N = J.N, K = J.K;
  const int nt = gram_tiles(T), npair = nt * (nt + 1) / 2;
  if ((int)blockIdx.x >= npair * nsb) return;         // block-uniform
  const int pair = blockIdx.x / nsb, sb = blockIdx.x - pair * nsb;
  const int wave = threadIdx.x >> 6, nslice = nsb * GB_WAVES, sl = sb * GB_WAVES + wave;
  int ta = 0, rem = pair;                              // upper triangle: (ta, tb), ta <= tb
  while (rem >= nt - ta) { rem -= nt - ta; ++ta; }
  const int tb = ta + rem;
  const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  const bool cond = J.h != nullptr;
  // this lane's rows: s = 0, 1 the A side (16-row blocks of tile ta), s = 2, 3 the B side (tb)
  int row[4];
  bool rok[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int t = (s < 2 ? ta : tb) * 32 + 16 * (s & 1) + r;
    rok[s] = t < T;
    row[s] = rok[s] ? t : T - 1;
  }
  f64x4 gc[2][2], gu[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) { gc[x][y] = f64x4{0, 0, 0, 0}; gu[x][y] = f64x4{0, 0, 0, 0}; }
  const auto Rm = gp(J.Rm);
  const auto invT = gp(J.invT);
  if (cond) {
    // inner axis: e = i*K + k in 16-element chunks, split evenly over the slices
    // (32-bit index math: N * K < 2^31, checked by the launcher; a 64-bit division per chunk
    // was a large share of the VALU work)
    const int E = N * K;
    const int nch = (E + 15) / 16;
    const int c0 = (int)((long)nch * sl / nslice), c1 = (int)((long)nch * (sl + 1) / nslice);
    const unsigned uK = (unsigned)K;
    const auto h = gp(J.h);
    // two register batches of GB_U chunks: the loads of the next batch are in flight while the
    // MFMAs of this one run (the single-batch loop spent ~40% of its cycles waiting on memory:
    // SQ_WAIT_INST_ANY, profiles/r4_pmc_summary.txt). Same accumulation order as one batch.
    struct Batch {
      f32x4 hv[GB_U][4];
      float rm[GB_U][4], iv[GB_U];
    };
    auto load = [&](int cb, Batch& B) {
#pragma unroll
      for (int u = 0; u < GB_U; ++u) {
        const int e = (cb + u) * 16 + 4 * q;
        const bool eok = cb + u < c1 && e < E;
        const unsigned ec = eok ? (unsigned)e : 0u;
        const int i = (int)(ec / uK);
        B.iv[u] = eok ? invT[i] : 0.f;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          B.hv[u][s] = ld4(h + (size_t)row[s] * E + ec);
          B.rm[u][s] = rok[s] ? Rm[(size_t)row[s] * N + i] : 0.f;
        }
      }
    };
    auto comp = [&](const Batch& B) {
#pragma unroll
      for (int u = 0; u < GB_U; ++u) {
        double a[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) a[s] = (double)B.rm[u][s] * (double)B.iv[u];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          double va[2], vb[2];
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            va[s] = (double)B.hv[u][s][j] * a[s];
            vb[s] = (double)B.hv[u][2 + s][j] * a[2 + s];
          }
#pragma unroll
          for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) gc[x][y] = mfma_f64(va[x], vb[y], gc[x][y]);
        }
      }
    };
    Batch b0, b1;
    if (c0 < c1) load(c0, b0);
    for (int cb = c0; cb < c1; cb += 2 * GB_U) {
      if (cb + GB_U < c1) load(cb + GB_U, b1);
      comp(b0);
      if (cb + GB_U >= c1) break;
      if (cb + 2 * GB_U < c1) load(cb + 2 * GB_U, b0);
      comp(b1);
    }
  }
  {
    // Gu (both modes): inner axis = stocks, 4 per MFMA (k-slot q <-> stock 4c + q) -- dense
    // operands, an eighth of the MFMAs of riding along Gc's (stock, moment) chunks
    const int nch = (N + 3) / 4;
    const int c0 = (int)((long)nch * sl / nslice), c1 = (int)((long)nch * (sl + 1) / nslice);
    for (int cb = c0; cb < c1; cb += GB_U) {
      float rm[GB_U][4], iv[GB_U];
#pragma unroll
      for (int u = 0; u < GB_U; ++u) {
        const int i = 4 * (cb + u) + q;
        const bool iok = cb + u < c1 && i < N;
        const int ic = iok ? i : 0;
        iv[u] = iok ? invT[ic] : 0.f;
#pragma unroll
        for (int s = 0; s < 4; ++s) rm[u][s] = rok[s] ? Rm[(size_t)row[s] * N + ic] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < GB_U; ++u) {
        double a[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) a[s] = (double)rm[u][s] * (double)iv[u];
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int y = 0; y < 2; ++y) gu[x][y] = mfma_f64(a[x], a[2 + y], gu[x][y]);
      }
    }
  }
  // fixed-order sum of the block's slices in LDS (one 32x32 tile of Gc and Gu), then one store.
  // C/D map of v_mfma_f64_16x16x4_f64: lane l, register g -> row (l >> 4) + 4 g, column l & 15.
  __shared__ double acc[2][2][2][4][64];               // [c/u][x][y][g][lane]
  for (int w = 0; w < GB_WAVES; ++w) {
    if (wave == w) {
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            acc[0][x][y][g][lane] = (w ? acc[0][x][y][g][lane] : 0.0) + gc[x][y][g];
            acc[1][x][y][g][lane] = (w ? acc[1][x][y][g][lane] : 0.0) + gu[x][y][g];
          }
    }
    __syncthreads();
  }
  const size_t T2 = (size_t)T * T;
  const auto out = gp(J.part) + (size_t)sb * 2 * T2;
  for (int idx = threadIdx.x; idx < 2 * 2 * 2 * 4 * 64; idx += 64 * GB_WAVES) {
    const int l = idx & 63, g = (idx >> 6) & 3, y = (idx >> 8) & 1, x = (idx >> 9) & 1, c = idx >> 10;
    const int t = ta * 32 + 16 * x + (l >> 4) + 4 * g;
    const int u = tb * 32 + 16 * y + (l & 15);
    if (t < T && u < T) out[(size_t)c * T2 + (size_t)t * T + u] = (c == 0 && !cond) ? 0.0 : acc[c][x][y][g][l];
  }
}

// Sum the slices (fixed order) and mirror: G[w][t][u] for every t, u (from the tile holding
// min/max of the pair). grid (ceil(T*T / 256), jobs).
__global__ __launch_bounds__(256) void k_gram_reduce(const GramJob* __restrict__ jobs, int nslice) {
  const GramJob& J = jobs[blockIdx.y];
  const int T = J.T;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)T * T) return;
  const int t = (int)(e / T), u = (int)(e - (long)t * T);
  const int ta = t >> 5, tb = u >> 5;
  // the upper-triangle tile (by 32-row tile index) holds the element; inside a diagonal tile
  // both orders were written
  const int a = ta <= tb ? t : u, b = ta <= tb ? u : t;
  const size_t T2 = (size_t)T * T, src = (size_t)a * T + b;
  const auto part = gp(J.part);
  double sc = 0.0, su = 0.0;
  // RB slices' loads in flight before the (in-order) adds: one memory round trip per RB slices
  // instead of one per slice (same summation order)
  constexpr int RB = 16;
  for (int s0 = 0; s0 < nslice; s0 += RB) {
    double pc[RB], pu[RB];
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const size_t o = (size_t)min(s0 + k, nslice - 1) * 2 * T2 + src;
      pc[k] = part[o];
      pu[k] = part[o + T2];
    }
#pragma unroll
    for (int k = 0; k < RB; ++k)
      if (s0 + k < nslice) {
        sc += pc[k];
        su += pu[k];
      }
  }
  gp(J.G)[e] = sc;
  gp(J.G)[T2 + e] = su;
}

// workgroups per tile (each GB_WAVES slices of the inner axis): ~256 workgroups per model
// (DLAP_GRAM_WG; fewer slices leave CUs to the head epoch that the evaluation-split builds
// overlap and shrink the reduce pass: profiles/r3_knobs_gram_grid.log). A function of T only:
// the split-K partition -- and so the bits of G -- must not depend on how many models share
// the launch.
int gram_slices(int T) {
  static const int target = [] { const char* v = std::getenv("DLAP_GRAM_WG"); return v ? std::atoi(v) : 256; }();
  const int nt = (T + 31) / 32, npair = nt * (nt + 1) / 2;
  const int want = target / std::max(1, npair);
  return std::max(1, std::min(64, want));
}

size_t gram_part_doubles(int T, int njobs) {
  return (size_t)njobs * gram_slices(T) * 2 * (size_t)T * T;
}

void launch_gram(const GramJob* jobs, int njobs, int T, int nslice, hipStream_t st) {
  if (njobs <= 0 || T <= 0) return;
  const int nt = (T + 31) / 32, npair = nt * (nt + 1) / 2;
  hipLaunchKernelGGL(k_gram_build, dim3(npair * nslice, njobs), dim3(64 * GB_WAVES), 0, st, jobs, nslice);
  HIP_OK(hipGetLastError());
  hipLaunchKernelGGL(k_gram_reduce, dim3((unsigned)(((long)T * T + 255) / 256), njobs), dim3(256), 0, st, jobs,
                     nslice);
  HIP_OK(hipGetLastError());
}
