// Sparse-feature path of the fused encoder (see bgcn_sparse.hip).
#pragma once

#include "bgcn_internal.h"

namespace bgcn {

constexpr int kCap = 32;     // max non-zeros per feature row on the sparse path
constexpr int kChunk = kChunkItems;  // nodes per tree work item (conv2, dW2 root partials)

struct SparseState {
  int mode;        // 0 auto, 1 dense (sparse kernels idle), 2 sparse preferred (same as auto)
  int64_t N, F, B;
  // saved with the activations (caller-owned)
  int32_t* flags;  // [0] = some row has > kCap non-zeros -> dense path
  int32_t* nnz;    // [N]
  int32_t* cols;   // [N][kCap]
  float* vals;     // [N][kCap]
  // step scratch
  float* w1t;      // [F][128]     = [W1_td ; W1_bu]^T
  float* w2t;      // [2][64+F][64] = W2_d^T
  int max_items;
  int32_t *item_tree, *item_chunk, *tree_item0;
  float* root_part;  // [2][max_items][kCap][64]
  int32_t* hist;        // [R][F] per-row-block column counts -> prefixes (R = N / kRowBlock)
  int32_t* col_total;   // [F]
  int32_t *col_start, *col_end;  // [F]
  uint32_t* csc_slot;   // [N*kCap] slots (i*kCap + s) grouped by column, rows in order
  uint32_t* rbits;      // [2][N] forward's root keep masks (bit s: root non-zero s kept)
  float* csc_val;       // [N*kCap] X value of each csc_slot entry
  int32_t* zero_word = nullptr;   // zeroed by the prologue (the train step's status word)
};

constexpr int kRowBlock = kCscRowBlock;   // rows per block of the CSC counting sort
constexpr int64_t kSparseMaxF = kSparseMaxFeat;  // LDS bound of the CSC kernels (2 x 4 B x F)

size_t carve_sparse(Carve& c, int64_t N, int64_t B, int64_t F, SparseState* S);
// forward prologue: weight transposes (sparse path), node_root, tree_ptr, flag reset
// batch_part = false: weight transposes only (the batch part came from a Prepared)
int sparse_prologue(SparseState& S, const bgcn_bigcn_args* a, int32_t* node_root, hipStream_t s,
                    bool batch_part = true);
struct Prepared;
// weight-independent preparation of one batch into p (bgcn_prepare_batch)
int sparse_prepare(const Prepared& p, int64_t N, int64_t B, int64_t F, int mode,
                   const int64_t* batch, const int64_t* rootindex, const void* X, int xdt, int64_t ldx,
                   hipStream_t s);
int sparse_conv1_gather(SparseState& S, float* Z1, hipStream_t s);
int sparse_compact_conv1(SparseState& S, const void* X, int xdt, int64_t ldx, float* Z1,
                         hipStream_t s);
int sparse_items(SparseState& S, const int32_t* tree_ptr, hipStream_t s);
int sparse_conv2(SparseState& S, const float* H1, const int32_t* tree_ptr, const int64_t* rootindex,
                 float* Z2, KeepSrc keep, hipStream_t s);
int sparse_csc(SparseState& S, hipStream_t s);
int sparse_dw2_root_part(SparseState& S, const int32_t* tree_ptr, const float* dZ2, hipStream_t s);
int sparse_dw1(SparseState& S, const bgcn_bigcn_args* a, const float* dZ1, hipStream_t s,
               const ColsumJob& job);
int sparse_dw2_rootcols(SparseState& S, const bgcn_bigcn_args* a, const int32_t* node_root,
                        KeepSrc keep, hipStream_t s);

}  // namespace bgcn
