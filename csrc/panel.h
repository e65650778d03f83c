// Device-side split preparation (k_panel.hip): the compacted engine layout of a dense split
// built on the GPU, with no host round trip of the panel.
#pragma once
#include <stdint.h>
#include "common.h"

struct PanelIn {           // a dense split in device memory (the caller's tensors)
  const float* feats;      // [T][N][F] characteristics (nullptr: statistics only)
  const float* ret;        // [T][N] returns (any value where the mask is 0)
  const uint8_t* maskb;    // [T][N] bool mask, or
  const float* maskf;      // [T][N] 0/1 float mask (when maskb is null)
  int T, N, F;
};

struct PanelOut {
  float* Rm;               // [T*N] returns, zero where masked (written unless Rm_in_place)
  float* mask;             // [T*N] 0/1
  float* Nt;               // [T] valid stocks of each period
  float* invNt;            // [T] 1 / max(N_t, 1)
  float* meanR;            // [T] sum_i R m / max(N_t, 1)   (double accumulation)
  float* RR;               // [T] sum_i R^2 m                (double accumulation)
  float* invT;             // [N] 1 / max(T_i, 1)
  int* cnt;                // [T] scratch: N_t as int
  int* row_ptr;            // [T+1] first compact row of each period
  float* nbar;             // [1] mean_t max(N_t, 1) (fp32 of a double sum, as the host did)
  int2* rowti;             // [R] (t, i) of each compact row, (t, i) order
  float* Rc;               // [R] returns of the compact rows
  uint16_t* X;             // [R][KP] bf16 rows (fp32: [R][2 KP] uint16 = [R][KP] float)
  int KP;
  int fp32;
  int dense_out;           // 1: write Rm / mask (0: they are the inputs already)
};

// counts, dense Rm / mask, per-period sums, per-asset counts, row_ptr and N-bar
void launch_panel_stats(const PanelIn& in, const PanelOut& out, hipStream_t st);
// rowti, Rc and the feature rows X of the R = row_ptr[T] valid rows (after launch_panel_stats)
void launch_panel_compact(const PanelIn& in, const PanelOut& out, int R, hipStream_t st);
