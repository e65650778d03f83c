// Model descriptor shared by the host engine and the kernels.
//
// Flat fp32 parameter vector = the reference module's state_dict() order
// (ModelSpec.param_layout in config.py): LSTM (w_ih, w_hh, b_ih, b_hh per layer), SDF fc
// layers (W, b)..., SDF output (w, b), moment fc layers (W, b)..., moment output (W, b).
// [0, P_sdf) is sdf_net, [P_sdf, P) is moment_net.
//
// The tower kernels never read the flat vector: after every optimiser step the update
// kernel re-packs the weights into a bf16 "blob" of MFMA operand fragments (1 KiB per
// 16x32 fragment = 64 lanes x 8 bf16, lane-linear, so staging it in LDS and reading one
// ds_read_b128 per lane is bank-conflict free) plus an fp32 "aux" vector (biases, output
// row, per-period column weights). Fragment maps: k_mlp.hip header.
#pragma once
#include "mlp.h"

#define DLAP_MAX_RNN 4       // max LSTM layers
#define DLAP_MAX_H 32        // max LSTM width

struct PackLayer {
  int w_off, b_off;   // flat offsets of W [out][ld] and b [out]
  int out, in;        // true widths (layer 0: number of X-tile columns that map to W)
  int ld, col0;       // row stride of W; flat column of X-tile column 0
};

// One weight-gradient tile of 64 outputs x 64 inputs: (tower layer, 64-column chunk).
struct GradTile {
  int w_off, ld, col0;      // flat mapping of element (o, 64*chunk + i)
  int out, in, chunk;
  int slice;                // slab slice that owns the tile
  int layer;                // tower layer (> 0: the packed training weights carry the dropout
                            //   scale, so the gradient is scaled back by k_finalize)
  int xmap;                 // 1: fused SDF layer 0 -- i is a panel column: [0, F) -> W0 column i,
                            //   [ppc, ppc + Dm) -> W0 column F + i - ppc, else no weight
};

#define DLAP_MAX_TILES 16

struct ModelDesc {
  // dimensions
  int F, M, Dm, KIN, KP, KS1, WMB;
  int KSB;                  // layer-0 k-steps packed into the tower blob (KS1; 0 on the wide path)
  int K, cm1;
  int nrnn, H;
  int P, P_sdf;
  float dropout;
  int normalize_w, weighted_loss;
  float residual_factor;
  // flat parameter map
  int lstm_w_ih[DLAP_MAX_RNN], lstm_w_hh[DLAP_MAX_RNN], lstm_b_ih[DLAP_MAX_RNN], lstm_b_hh[DLAP_MAX_RNN];
  int nl_s, nl_m;
  PackLayer s[DLAP_MAXL];   // SDF hidden layers
  int so_w, so_b;           // SDF output_proj weight [1][hs_last], bias [1]
  PackLayer m[DLAP_MAXL];   // moment layers; m[0] spans [macro ; x] (ld = M + F)
  // packed blob / aux offsets (also in md)
  MlpDims md;
  // gradient reduction tables (phase-specific tower)
  int ntile_s, ntile_m, nslice_s, nslice_m;
  int tps_s, tps_m;        // gradient tiles accumulated per backward slice
  int tbwd;                 // 1: the SDF backward is the one-pass k_tbwd_sdf (k_tbwd.hip; one slice,
                            //   tps_s = ntile_s), else the sliced k_mlp_bwd_sdf
  // input-projection matrix re-packed by k_pack for k_proj: wproj[MP + 2][NP] fp32, row m < M =
  // column m of [W_ih(layer 0) ; W_m0[:, :M]], row MP = (b_ih ; b_m0), row MP + 1 = (b_hh ; 0)
  int proj_mp, proj_np;
  GradTile tile_s[DLAP_MAX_TILES], tile_m[DLAP_MAX_TILES];
  int extra_s[SLAB_EXTRA], extra_m[SLAB_EXTRA];   // slab extra slot -> flat index (-1 unused)
};
