// Job record of the loss / metric kernels (k_loss.hip), shared with the engine.
#pragma once
#include <vector>
#include "common.h"

#define DLAP_MAX_T 2048   // max periods per split handled by the LDS-staged passes
#define DLAP_TCH 8        // time chunks of the asset pass

// Scalar slots written per job by k_job_metrics.
enum {
  SC_LCOND = 0, SC_LUNC = 1, SC_LRES = 2, SC_TRAIN_SHARPE = 3,
  SC_SHARPE = 4, SC_MEAN = 5, SC_STD = 6, SC_MDD = 7, SC_NSCAL = 8
};

struct LossJob {
  // panel constants of the split
  const float* Rm;       // [T*N] returns, zero at invalid entries
  const float* mask;     // [T*N] 0/1
  const float* invNt;    // [T] 1 / max(N_t, 1)
  const float* Nt;       // [T] N_t
  const float* meanR;    // [T] sum_i R m / max(N_t, 1)
  const float* RR;       // [T] sum_i R^2 m
  const float* invT;     // [N] 1 / max(T_i, 1)
  const int* row_ptr;    // [T+1] compact rows of each period
  const int2* rowti;     // [R] (t, i) of each compact row
  const float* Rc;       // [R] returns of the compact rows
  float* mu;             // [T] cross-sectional mean of the raw weights
  float Nbar;
  int T, N, K;
  int R;                 // compact rows of the split (bounds of w / Rc / rowti / dw)
  int normalize, weighted;
  int phase;             // 1: unconditional, 2: moment, 3: conditional, 0: evaluation
  float res_factor;      // residual_loss_factor (gradient only in training jobs)
  float coef_c, coef_u;  // dL/dE = coef * E (0 disables the write)
  int asset_full;        // 1: one-pass asset reduction (k_asset_full), else k_asset_part + k_asset_red
  // per (model, split) workspace
  const float* w;        // [R] raw SDF output (compact rows)
  float* wn;             // [T*N] normalised weights w' (dense, zero at invalid entries)
  const float* h;        // [T*N*K] moments (nullptr: unconditional only)
  float* P;              // [T] weighted portfolio return
  float* port;           // [T] L1-normalised portfolio return (nullptr: skip)
  float* sdfv;           // [T] 1 + P_t
  float* E;              // [N*K]
  float* Eu;             // [N]
  float* dE;             // [N*K] (nullptr: skip)
  float* dEu;            // [N]   (nullptr: skip)
  float* part;           // [2 * ceil(N (K+1) / 256)] partial loss sums
  float* pe;             // [DLAP_TCH][N][K] chunk partials of E
  float* pu;             // [DLAP_TCH][N] chunk partials of E_unc
  float* dw;             // [R] dL/dw_raw (compact rows)
  float* rstat;          // [T*4] residual statistics (nullptr: residual loss off)
  float* scal;           // [SC_NSCAL]
  // Gram mode (k_gram.hip; moments frozen): the loss is the quadratic form s^T G s, so the
  // asset passes are skipped and k_period_bwd evaluates G s per period. h is then only a flag
  // (non-null: the conditional loss is wanted) and E / dE are not produced.
  int gram;              // 1: Gram mode
  const double* G;       // [2][T][T] Gc, Gu
  double* gpart;         // [T][2] per-period s_t (G s)_t of Gc and Gu
  int* prog_reset;       // train jobs: the fused forward's progress counter of this (model, split),
                         //   zeroed by k_period_fwd (it follows every fused forward; nullptr: none)
  // Cross-sectional sharding (parallel/xsection.py, the engine path): this engine holds one rank's
  // stocks. Every cross-sectional sum is formed locally, summed over the ranks between launches
  // (the engine's hook) and consumed from here; the per-period constants (N_t, mean R, Nbar) are
  // the global ones and Nnorm is the global stock count of the loss means.
  float* xs;             // [4][T] per-period partial sums (nullptr: not sharded), then [2] the
                         //   phase-2 / dense-evaluation loss sums
  float Nnorm;           // N of the loss normalisation (J.N unless sharded)
};

// One (model, split) of the Gram build (k_gram.hip).
struct GramJob {
  const float* h;        // [T*N*K] frozen moments (nullptr: only Gu)
  const float* Rm;       // [T*N] returns, zero at invalid entries
  const float* invT;     // [N]
  double* part;          // [nslice][2][T][T] split-K partials (scratch)
  double* G;             // [2][T][T] out: Gc, Gu
  int T, N, K;
};
int gram_slices(int T);
size_t gram_part_doubles(int T, int njobs);
// all jobs of one launch share T (one split of every model)
void launch_gram(const GramJob* jobs, int njobs, int T, int nslice, hipStream_t st);

// store_wn = false: the epoch graphs (nothing in the epoch reads the dense zero-mean weights)
// stage (sharded jobs, LossJob::xs): 1 the local sum of the raw weights per period -> xs[0]; 2 with
// the global sum back in xs[0]: the zero-mean weights' local sums sum w'R, sum |w'|, sum w'^2 ->
// xs[1..3]; 3 with those global: P, SDF, the L1 portfolio return, the residual statistics.
// 0: all of it from the local rows (one launch).
void launch_period_fwd(const LossJob* jobs, int njobs, int tmax, hipStream_t st, bool store_wn = true,
                       int stage = 0);
// sharded jobs: the local loss sums of the asset passes (sum E^2 over k, i and sum E_u^2) ->
// xs[4 T], xs[4 T + 1]; once summed over the ranks k_job_metrics takes them from there
void launch_xs_loss_sums(const LossJob* jobs, int njobs, hipStream_t st);
// kmax: the moment count K of the jobs (sizes the output grid of the reduction pass)
// full: the one-pass k_asset_full (training jobs: fewer launches on the critical chain; the
// jobs must have been built with asset_full = 1), else k_asset_part + k_asset_red (evaluation
// jobs: more parallel over the long test split, off the critical chain)
void launch_asset(const LossJob* jobs, int njobs, int nmax, int kmax, hipStream_t st, bool full = false);
// metrics: also compute the job metrics (k_job_metrics) in one extra workgroup
void launch_period_bwd(const LossJob* jobs, int njobs, int tmax, hipStream_t st, bool metrics = false);
bool asset_full_default();   // DLAP_ASSET_FULL (default 1): one-pass asset reduction for training jobs
void launch_job_metrics(const LossJob* jobs, int njobs, hipStream_t st);
std::vector<long long> loss_timestamps();
// ensemble averaging + re-normalisation + portfolio returns (K11), device pointers
void launch_ensemble(const float* W, int G, int T, int N, const float* R, const float* mask, float* port,
                     float* port_ind, hipStream_t st);
