// Job records of the gradient-finalise / optimiser / bookkeeping kernels (k_update.hip).
#pragma once
#include "common.h"

struct ModelDesc;

#define PACK_FAN 4
#define ADAM_PB 1024          // parameters per Adam block (adam_block, k_adam, the tail's Adam blocks)
// hand-off words of the fused backward tail (UpdJob::tail_ctr, 128 bytes apart): the per-period
// sums published, the gate-gradient flag, the W_ih blocks done, the blocks arrived (Adam in the
// tail, a running count) and the evaluation branch's signals (a running count)
#define TAIL_CNT 0
#define TAIL_FLAG 32
#define TAIL_DONE 64
#define TAIL_ARRIVE 96
#define TAIL_EVGEN 128
#define TAIL_ARRIVE2 160       // (phase-2 tail launches: their own running arrival count)
#define TAIL_ADONE 192         // tail Adam blocks finished (running count)
#define TAIL_UPDGEN 224        // tail updates finished (running count; the last Adam block of a launch)
#define TAIL_UPDSEEN 256       // updates the evaluation graph has consumed (k_wait_gen)
#define TAIL_WORDS 288         // max packed copies of one parameter for k_adam's fused re-pack

struct FinJob {            // one model
  const float* slab;       // first slab of this model (slices contiguous, gx slabs each)
  float* grads;            // flat gradient vector [P]
  const int* row_ptr;      // [T+1] compact-row offsets of the train split
  const float* u;          // [R][Dm] per-row d(per-period SDF input)
  float* dpp;              // [T][Dm]
  const float* v;          // [R][64] per-row d(moment layer-0 pre-activation)
  float* dab;              // [T][64]
  int T;
  float dropout;           // the model's dropout rate (gradients of scaled weights are scaled back)
  int nslab;               // slabs stored per slice
  int group;               // 4: they are fine slabs, summed in groups of 4 first; 1: coarse slabs
};

struct UpdJob {            // one model
  float* params;
  float* grads;
  float* m;                // Adam first moments [P]
  float* v;                // Adam second moments [P]
  int* adam_step;          // [2] optimiser step counts (sdf, moment)
  int* drop_step;          // dropout stream counter
  float* gnorm;            // [1] pre-clip gradient norm of the step
  bf16x8* blob;
  bf16x8* blob0;           // wide path: layer-0 x-column fragments of k_proj0 (nullptr: none)
  float* aux;
  float* wproj;            // packed input-projection matrix (written by k_pack)
  const float* dpp;        // [T][Dm] d(LSTM output)
  const float* macro;      // [T][M] train macro series
  const float* sg;         // [nrnn][T][4H] saved post-activation gates
  const float* sc;         // [nrnn][T][H]  saved cells
  const float* sh;         // [nrnn][T][H]  saved layer outputs
  float* dg;               // scratch [T][4H]
  float* dx;               // scratch [T][H]
  const float* dab;        // [T][64]
  const float* h0;         // [nrnn][H] initial LSTM state of the train split (zero by default)
  const float* c0;
  float* dh0;              // [nrnn][H] out: dL/d(initial state) (module API: a caller's hidden)
  float* dc0;
  const float* scal;       // train-split job scalars of this step (SC_NSCAL) ...
  float* scal_prev;        // ... copied here by k_adam for the epoch bookkeeping
  int T;
  unsigned seed;
  float dropout;           // the model's dropout rate (k_pack folds 1/(1-p) into the train blob)
  float lr;                // > 0: this model's learning rate (sweeps batch configs that
                           // differ only in lr); 0: the launch-wide lr
  const int* prog;         // the model's fused-forward progress records (3 splits, 16 ints each;
                           // [16 s + 1] = spin waits that gave up): non-zero poisons the model --
                           // k_adam skips every later update, k_epoch_end records NaN epochs
  const int* inv_code;     // [P][PACK_FAN] scatter lists: the packed elements holding parameter p
                           // (-1 padded; nullptr: a separate k_pack re-packs after k_adam)
  int* upd_ctr;            // [1] k_adam blocks finished (the last one advances the step counters)
  int* tail_ctr;           // fused backward tail (k_lstm_tail): per-period sums published so far
                           //   (zero between launches: the LSTM block rearms it)
  float* mscr;             // fused backward tail: [T][64] LSTM step-matrix scratch (train split)
  unsigned spin_limit;     // fused backward tail: polls before the wait for dpp gives up
};

// History row written per epoch by k_epoch_end (HIST_W floats).
enum {
  H_PHASE = 0, H_TRAIN_LOSS, H_TRAIN_SHARPE, H_VALID_LOSS, H_VALID_SHARPE, H_TEST_LOSS,
  H_TEST_SHARPE, H_TRAIN_LUNC, H_TRAIN_LCOND, H_GNORM, H_VALID_LUNC, H_VALID_LCOND,
  H_VALID_MDD, H_VALID_MEAN, H_VALID_STD, H_TEST_LUNC, H_TEST_LCOND, H_TEST_MDD,
  H_TEST_MEAN, H_TEST_STD, H_TRAIN_LRES, H_BEST_LOSS, H_BEST_SR, H_SNAP, HIST_W = 24
};

struct EpochJob {          // one model
  const float* sc_train;   // job scalars (SC_*) of the train job
  const float* sc_valid;   // nullptr in phase 2
  const float* sc_test;    // nullptr if no test split / phase 2
  const float* gnorm;
  float* hist;             // [max_epochs][HIST_W]
  int* ep;                 // [2] global epoch index, epoch within the phase
  float* best;             // [3] best valid loss, best (signed) valid Sharpe, best moment loss
  int* snap_flags;         // [2] loss snapshot taken, Sharpe snapshot taken (this phase)
  const float* params;
  float* snap_loss;        // [P]
  float* snap_sharpe;      // [P]
  int max_ep;              // rows of hist: epochs past the capacity are not recorded
  const int* prog;         // as UpdJob::prog (a poisoned model records NaN epochs, no snapshots)
  int* eval_gen;           // the model's tail_ctr + TAIL_EVGEN: bookkeeping launches that signal
                           // (the pipelined epoch's evaluation branch) count here when done
};

void launch_finalize(const FinJob* jobs, int njobs, const ModelDesc* md, const ModelDesc& mh,
                     int phase, int slab_stride, int tmax, hipStream_t st, int part = 0);
// fused: the jobs carry scatter lists (UpdJob::inv_code) -- k_adam re-packs, no k_pack launch
void launch_update(const UpdJob* jobs, int njobs, const ModelDesc* md, const ModelDesc& mh, int phase,
                   float lr, hipStream_t st, bool fused);
void launch_lstm_bwd(const UpdJob* jobs, int njobs, const ModelDesc* md, const ModelDesc& mh,
                     int T, int phase, hipStream_t st);
// fused backward tail of phases 1 / 3: k_finalize + k_lstm_bwd + k_wgrad as one launch (k_rnn.hip)
bool lstm_tail_supported(const ModelDesc& mh, int T);
int lstm_tail_words();     // ints of UpdJob::tail_ctr (hand-off words, 128 bytes apart)
// workgroups of k_lstm_tail the device holds at once (occupancy query x CUs) at split length T
int lstm_tail_capacity(const ModelDesc& mh, int T);
struct LossJob;
// ljobs: the train split's loss jobs whose job metrics one more block per model computes (or nullptr)
// adam: 0 = none (k_adam follows); 2 = the update runs in the tail (the launch's last blocks,
// adam_block) after the epoch's evaluation branch signalled (launch_epoch_end); 1 = the same
// without that signal (phase 2: nothing else reads the parameters during the epoch); 3 = as 2, and
// the launch's last Adam block advances the model's update generation (k_wait_gen, DLAP_EVAL_SEP)
// phase 2: the moment network's tail -- k_finalize + k_wgrad (the macro columns of moment layer
// 0) [+ k_adam]; block 0 relays the per-period sums' count to the W_macro helpers (no BPTT)
void launch_lstm_tail(const UpdJob* ujobs, const FinJob* fjobs, int njobs, const ModelDesc* md, const ModelDesc& mh,
                      int T, int slab_stride, hipStream_t st, const LossJob* ljobs = nullptr, int adam = 0,
                      float lr = 0.f, int phase = 1);
// whether the phase-2 tail applies (macro columns in moment layer 0)
bool mom_tail_supported(const ModelDesc& mh, int T);
void launch_pack(float* const* params_unused, const UpdJob* jobs, int njobs, const ModelDesc* md,
                 const ModelDesc& mh, hipStream_t st);
int pack_total(const ModelDesc& mh);   // packed elements per model (k_pack's element space)
void pack_index_host(const ModelDesc& mh, int* src);   // packed element -> parameter (-1: padding)
void launch_set_int(int* p, int v, hipStream_t st);
void launch_begin_phase(const EpochJob* jobs, int njobs, hipStream_t st);
// the split epoch graphs' evaluation graph waits (one wave) for `per` more finished evaluation
// recurrences of the training graph's fused forward than it consumed so far (cnt[0] running
// count, cnt[32] consumed); giving up poisons the nmodels models (prog records, 48 ints each)
void launch_wait_count(int* cnt, int per, unsigned limit, int* prog, int nmodels, hipStream_t st);
// the split epoch graphs with the evaluation recurrences on the evaluation queue: the evaluation
// graph's first launch waits (one wave) until every model's previous update is complete (the
// tail's TAIL_UPDGEN one past TAIL_UPDSEEN), then consumes it; giving up poisons the models.
// launch_gen_sync (after the head epoch's k_adam, which does not count): the next wait passes.
void launch_wait_gen(const UpdJob* jobs, int njobs, unsigned limit, hipStream_t st);
void launch_gen_sync(const UpdJob* jobs, int njobs, hipStream_t st);
// signal: each model's block counts its EpochJob::eval_gen when done (agent release) -- the
// fused tail's Adam blocks wait for it (launch_lstm_tail, adam 2)
void launch_epoch_end(const EpochJob* jobs, int njobs, int phase, int ignore_epoch, float sel,
                      float res_factor, int P, hipStream_t st, int signal = 0);
