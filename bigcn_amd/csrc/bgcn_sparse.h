// Sparse-feature path of the fused encoder (see bgcn_sparse.hip).
#pragma once

#include "bgcn_internal.h"

namespace bgcn {

constexpr int kCap = 32;     // non-zeros per feature row held in the ELL list
// A row of more than kCap non-zeros keeps its first kCap in the ELL list and spills the
// rest, in column order, to a per-batch pool of (col, value bits) pairs (kSpillPerRow
// entries per row of capacity: a batch may hold N * (kCap + kSpillPerRow) non-zeros).
// Every product with X is a sum over non-zeros, so the spilled entries add their terms
// in extra loops of the same kernels; only a batch whose spill exceeds the pool falls
// back to the dense MFMA path.
constexpr int kSpillPerRow = BGCN_SPARSE_SPILL_PER_ROW;
constexpr int kW2sLd = 64 + kCap + 8;   // bf16 row strides of the split W2 images (16-byte
constexpr int kW2dLd = 64 + 8;          // aligned rows; conv2's also holds 32 root slots)
constexpr int kChunk = kChunkItems;  // nodes per tree work item (conv2, dW2 root partials)

struct SparseState {
  int mode;        // 0 auto, 1 dense (sparse kernels idle), 2 sparse preferred (same as auto)
  int64_t N, F, B;
  // saved with the activations (caller-owned)
  int32_t* flags;  // [0] = the batch's spill exceeds the pool -> dense path; [1] = pool fill;
                   // [2] = rows over kCap (long_rows)
  int32_t* nnz;    // [N]
  int32_t* cols;   // [N][kCap]
  float* vals;     // [N][kCap]
  int32_t* ovf_off;   // [N] first pool entry of row i (valid when nnz[i] > kCap)
  int32_t* long_rows; // [N] the rows over kCap (count in flags[2]; conv1's long-row blocks)
  uint2* ovf;         // [ovf_cap] spilled (col, value bits), row by row, columns ascending
  int64_t ovf_cap;
  // step scratch
  float* w1t;      // [F][128]     = [W1_td ; W1_bu]^T
  float* w2t;      // [2][64+F][64] = W2_d^T
  // W2_d[:, :64] split for the bf16 MFMA once per step by the prologue (the blocks of
  // conv2 / the middle launch copy them instead of splitting per block):
  __bf16* w2s;     // [2][3][64 o][kW2sLd] hi / mid / lo of W2_d[o][k], k < 64 (conv2's B)
  __bf16* w2d;     // [2][3][64 c][kW2dLd] hi / mid / lo of W2_d[o][c] at [c][o] (dH1's B)
  int max_items;
  int32_t *item_tree, *tree_item0;
  int32_t *item_beg, *item_end, *item_root;   // item node range [beg, end), its tree's root
  float* root_part;  // [2][max_items][kCap][64]
  int32_t* hist;        // [R][F] per-row-block column counts -> prefixes (R = N / kRowBlock)
  int32_t* col_total;   // [F]
  int32_t *col_start, *col_end;  // [F]
  uint2* csc;           // [N*(kCap+kSpillPerRow)] (slot i*kCap + s, value bits) grouped by
                        // column, rows in order: one 8-byte store per placed entry (the
                        // placement scatters); a spilled entry's slot is i*kCap | kCscSpillFlag
  uint32_t* rbits;      // [2][N] forward's root keep masks (bit s: root non-zero s kept)
  int32_t* zero_word = nullptr;   // zeroed by the prologue (the train step's status word)
  int32_t* rtick = nullptr;       // [B] readout arrival counters, zeroed by the prologue
  int32_t* bstatus = nullptr;     // batch status word (bit 0: a batch id outside [0, B)), or nullptr
  const int32_t* root_map = nullptr;   // node -> its tree's root (the CSC placement flags root rows)
  int conv1_clears = 0;           // conv1's block 0 clears zero_word / rtick (no prologue launch)
  // per tree and direction, conv2's root-slot B operand (2 relu(x_root,col_s) W2_d^T[64 + col_s],
  // split three ways) built by extra blocks of conv1's launch (rimg_ready): conv2's fill then
  // copies it instead of walking root -> ELL slots -> W2^T rows
  __bf16* rimg = nullptr;         // [B][2][3][64 o][kCap] bf16
  uint32_t* rcols = nullptr;      // [B][kCap] H + col_s of the root's ELL slots (0 past nnz)
  int32_t* rinfo = nullptr;       // [B] the root row's non-zero count (ELL + spill)
  int rimg_ready = 0;
};
// The weight images of the sparse path in a caller-owned persistent buffer
// (bgcn_weight_images_size): kept current by bgcn_adam_step, so a step whose images are
// current launches no prologue (its transposes and splits were the Adam's tile epilogue).
struct WeightImages {
  float* w1t;      // [F][128]
  float* w2t;      // [2][F+64][64]
  __bf16* w2s;     // [2][3][64][kW2sLd]
  __bf16* w2d;     // [2][3][64][kW2dLd]
};
size_t carve_images(Carve& c, int64_t F, WeightImages* im);
// CSC slot bit 31: the entry's row is a tree root (its column gets a dW2 root-column term);
// bit 30: a spilled entry (no ELL slot; its root term is summed over the tree directly)
constexpr uint32_t kCscRootFlag = 0x80000000u;
constexpr uint32_t kCscSpillFlag = 0x40000000u;
constexpr uint32_t kCscSlotMask = 0x3fffffffu;
constexpr int64_t kSparseMaxN = int64_t(1) << 25;   // slots i*kCap below bit 30

constexpr int kRowBlock = kCscRowBlock;   // rows per block of the CSC counting sort
constexpr int64_t kSparseMaxF = kSparseMaxFeat;  // LDS bound of the CSC kernels (2 x 4 B x F)

size_t carve_sparse(Carve& c, int64_t N, int64_t B, int64_t F, SparseState* S);
// forward prologue: weight transposes (sparse path), node_root, tree_ptr, flag reset
// batch_part = false: weight transposes only (the batch part came from a Prepared)
int sparse_prologue(SparseState& S, const bgcn_bigcn_args* a, int32_t* node_root, hipStream_t s,
                    bool batch_part = true);
struct Prepared;
// weight-independent preparation of one batch into p (bgcn_prepare_batch)
// part 1: node maps, tree items, the ELL of X (the pass over X); part 2: the CSC of X
int sparse_prepare(const Prepared& p, int64_t N, int64_t B, int64_t F, int mode,
                   const int64_t* batch, const int64_t* rootindex, const void* X, int xdt, int64_t ldx,
                   hipStream_t s, int part = 3, const bgcn_batch* csr = nullptr);
// rootindex (optional): also build conv2's per-tree root images (SparseState::rimg) in the launch
int sparse_conv1_gather(SparseState& S, float* Z1, hipStream_t s, const int64_t* rootindex = nullptr,
                        float sc = 1.f);
int sparse_compact_conv1(SparseState& S, const void* X, int xdt, int64_t ldx, float* Z1,
                         hipStream_t s);
int sparse_items(SparseState& S, const int32_t* tree_ptr, const int64_t* rootindex, hipStream_t s);
int sparse_conv2(SparseState& S, const float* H1, const int32_t* tree_ptr, const int64_t* rootindex,
                 float* Z2, KeepSrc keep, hipStream_t s);
int sparse_csc(SparseState& S, hipStream_t s);
// The backward's middle and tail launches (bgcn_sparse.hip): role block counts the
// launchers fill in are marked (set by launcher).
struct Dw2Cfg {
  int64_t kchunk;
  int S, gx, want_dense;
  int64_t ldp;
  float* part;
};
struct RedCfg {
  int S;
  int64_t ldp;
  int want_dense;
  int blocks;   // 1024-thread blocks of this configuration in the launch
};
struct BwdMidArgs {
  SparseState S;                 // sizes (N, F, max_items), root partials (sparse)
  const void* X; int64_t ldx;
  const float *H1, *dZ2;
  const int32_t *node_root, *tree_ptr, *gate;
  KeepSrc keep;
  Dw2Cfg dw2_dense, dw2_sparse;  // dW2 partials: dense config blocks first
  int n_dw2_dense, n_dw2;
  int n_dw2b = 0, gxb = 0;        // dense mode, bf16 X: the root columns' blocks (k_dw2_bf16)
  int dw2b_f32 = 0;               // 1: k_dw2_root<float> (tree-run tiles, root factor per tile); 2: <bf16_t>
  int n_dw2h = 0;                 // the H1 columns' dw2_body blocks run first in that launch (not the middle one)
  int n_dw2f = 0;                 // dense mode, fp32 X: dw2_body's blocks as k_dw2_f32
  int n_root;                    // (set by launcher)
  const float *W2td, *W2bu;      // dH1
  float *dH1, *colpart;
  int nblk_h;                    // dH1 blocks per direction (node splits of rows_h nodes)
  int64_t rows_h;
  ColsumJob db2;
  const float* db2_dhead = nullptr;   // non-null: db2's partials are per-item positive-H2
                                      // counts (the readout-gradient aggregation, SpmmSign)
  HeadGradJob hg{};               // the classifier head's weight gradients (readout fused)
  int n_hg = 0;
};
struct BwdTailArgs {
  SparseState S;
  const float* dZ1;
  float *dw1_td, *dw1_bu;
  int n_dw1, n_rootcols;         // (set by launcher)
  const int32_t* node_root;
  const int64_t* batch;
  float *dw2_td, *dw2_bu;
  float keep_scale;
  KeepSrc keep;                  // spilled root entries: keep bits recomputed
  const float* dZ2;              // spilled root entries: summed over their tree
  const float* dw2_part;
  const int32_t* gate;
  RedCfg red_dense, red_sparse;
  ColsumJob db1;
  TailAdam adam;                 // the step's fused optimiser step (adam.on), part 0 only
};
int bwd_mid_launch(BwdMidArgs& a, int x_dtype, hipStream_t s);
int dw2_bf16_launch(BwdMidArgs& a, hipStream_t s);   // dense mode: dW2 root columns (bf16 MFMA)
int dw2_f32_launch(BwdMidArgs& a, hipStream_t s);    // dense mode, fp32 X: dW2 (k_dw2_f32)
// the whole weight-independent preparation of one batch on one stream (six launches;
// mode 1 = dense: no ELL / CSC of X); nlanes: 1 = every launch on `s`, 2 = DropEdge + K1
// forked onto the graph lane beside the pass over X, 0 = the default (BGCN_PREP_LANES)
int prep_pipeline(const Prepared& p, const bgcn_batch* b, int64_t F, int degree_on, int mode,
                  hipStream_t s, bool x_part = true, int nlanes = 0);
// part: 0 = the whole tail; 1 = all but dW1; 2 = dW1 only (the deferred-dW1 step)
int bwd_tail_launch(BwdTailArgs& a, hipStream_t s, int part = 0);

}  // namespace bgcn
