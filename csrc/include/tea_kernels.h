// Host-visible launcher interface of the torcheval_amd HIP kernels.
// Every launcher enqueues on the given HIP stream and returns hipError_t as int (0 = ok,
// -1 = unsupported argument combination, caller must fall back).
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include "tea_types.h"

namespace tea {

// ------------------------------------------------------------------ K1 classification
struct ClsCountsArgs {
  const void* input = nullptr;  // [n, c] scores (c > 0) or [n] integer labels (c == 0)
  DType in_dt = DType::f32;
  int64_t n = 0;
  int64_t c = 0;
  int64_t row_stride = 0;  // elements between rows of ``input``
  const void* target = nullptr;  // [n] integer labels
  DType tg_dt = DType::i64;
  int k = 1;                     // top-k (k > 1: rank-of-target)
  int64_t num_classes = 0;       // histogram width
  float* micro_correct = nullptr;
  float* micro_incorrect = nullptr;
  float* micro_total = nullptr;   // += n
  float* micro_total2 = nullptr;  // += n (second destination)
  float* cls_correct = nullptr;  // [num_classes] correct at target class
  float* cls_label = nullptr;    // [num_classes] samples per target class
  float* cls_pred = nullptr;     // [num_classes] samples per predicted class
  float* cls_fp = nullptr;       // [num_classes] wrong predictions per predicted class
  float* confusion = nullptr;    // [num_classes, num_classes] (target, pred)
  int* err = nullptr;            // error bits (1: bad target, 2: bad prediction)
  int* err_max = nullptr;        // optional [2]: largest target / prediction >= num_classes
  int check_target = 0;          // flag bad targets even without histograms
  unsigned long long* fold_ws = nullptr;  // tea_fold.h cells (per-stream, self-cleaning)
  // micro kernel only: per-wave correct counts go to these 64 pending cells (u64, 64-B stride)
  // instead of the fold into micro_correct; launch_micro_finish folds them later
  unsigned long long* pend = nullptr;
  int max_blocks = 0;
};
int launch_cls_counts(const ClsCountsArgs& a, hipStream_t stream);
// pending cells -> correct (+= their sum, cells zeroed); out = correct / total when given
constexpr int kPendCells = 64;
constexpr int kPendStride = 8;
int launch_micro_finish(unsigned long long* pend, float* correct, const float* total, float* out, hipStream_t stream);

struct BinaryCountsArgs {
  const void* input = nullptr;
  DType in_dt = DType::f32;
  const void* target = nullptr;
  DType tg_dt = DType::f32;
  const void* weight = nullptr;
  DType w_dt = DType::f32;
  int64_t n = 0;
  float threshold = 0.5f;
  int strict_binary = 0;  // non-{0,1} targets count nowhere (1) or as the "other" class (0)
  float* out[4] = {nullptr, nullptr, nullptr, nullptr};   // tp, fp, tn, fn
  float* out2[4] = {nullptr, nullptr, nullptr, nullptr};  // optional second destinations
  float* total = nullptr;  // += n (sample count)
  int max_blocks = 0;
};
int launch_binary_counts(const BinaryCountsArgs& a, hipStream_t stream);

// ------------------------------------------------------------------ K10 rank-of-target scores
struct RankArgs {
  const void* input = nullptr;  // [n, c] scores, unit column stride
  DType in_dt = DType::f32;
  int64_t n = 0;
  int64_t c = 0;
  int64_t row_stride = 0;
  const void* target = nullptr;  // [n] integer class index
  DType tg_dt = DType::i64;
  int mode = 0;  // 0: hit rate (rank < k), 1: reciprocal rank (0 beyond k when k > 0)
  int k = 0;
  float* out = nullptr;  // [n] float32 scores
  int* err = nullptr;    // bit 0: target out of range (row scored NaN)
};
int launch_rank_scores(const RankArgs& a, hipStream_t stream);

}  // namespace tea

namespace tea {

// ------------------------------------------------------------------ K3 sort-scan (AUROC/AUPRC)
struct AucScanArgs {
  int payload_kind = 0;  // 0: order = source index (gather); 1: order32 = f32 target bits; 2: order32 = class label
  const void* sorted = nullptr;  // [rows, n] scores sorted descending (f32 or f64)
  DType key_dt = DType::f32;
  int64_t key_stride = 0;
  const int64_t* order = nullptr;  // [rows, n] sort permutation (int64, torch.sort) ...
  const int32_t* order32 = nullptr;  // ... or int32 (K3a radix sort); exactly one is set
  int64_t order_stride = 0;
  const void* target = nullptr;  // binary: [rows, n] (row stride) / class mode: [n] labels
  DType tg_dt = DType::f32;
  int64_t target_stride = 0;
  const void* weight = nullptr;  // optional [rows, n]
  DType w_dt = DType::f32;
  int64_t weight_stride = 0;
  int class_mode = 0;  // positives are samples whose label == row index
  int64_t rows = 0;
  int64_t n = 0;
  double* out_auroc = nullptr;  // [rows]
  double* out_auprc = nullptr;  // [rows]
  // the onesweep sort's look-back timeout word of this stream (RadixArgs::os_hdr + 8) or null:
  // non-zero means the sort that produced `sorted` may have misplaced keys, and every output of
  // this scan is NaN instead of a wrong number
  const uint32_t* sort_fault = nullptr;
  // sample-sharded (distributed) mode: per-row (TP, FP) that precede this shard in the global
  // descending order, and raw sums [rows, 4] = (roc sum, pr sum, local P, local N) instead of
  // the normalised areas (the caller all-reduces them and normalises by the global P, N)
  const double* init = nullptr;  // [rows, 2]
  double* out_raw = nullptr;     // [rows, 4]
  // workspace carve-up (set by the launcher)
  void* ab = nullptr;
  void* tsum = nullptr;
  const void* tsum_ext = nullptr;  // [rows, ntiles] D2 tile totals already folded by the sort
  void* tstart = nullptr;
  void* tarea = nullptr;
  void* totals = nullptr;
  // K3c curve emission (PR curves / recall at fixed precision)
  int32_t* tcnt = nullptr;    // [rows, ntiles] tie-group tails per tile
  int32_t* cstart = nullptr;  // [rows, ntiles] exclusive scan of tcnt
  int64_t* sizes = nullptr;   // out [rows]: tie groups G_r (curve points without the final one)
  const int64_t* row_off = nullptr;  // [rows] threshold offset of row r (precision / recall: + r)
  float* out_prec = nullptr;  // [sum G_r + rows], ascending thresholds, final (1, 0) point per row
  float* out_rec = nullptr;
  void* out_thr = nullptr;    // [sum G_r], key dtype
  float min_precision = 0.f;  // RAFP mode
  float* s_rec = nullptr;     // [rows, n] recall per group (descending group order)
  void* s_thr = nullptr;      // [rows, n] threshold per group (key dtype)
  int32_t* gstar = nullptr;   // [rows] last group with precision >= min_precision (-1: none)
  int32_t* glo = nullptr;     // [rows] first group whose recall equals the maximum
  float* out_max_recall = nullptr;  // [rows]
  void* out_best_thr = nullptr;     // [rows], key dtype
};
int64_t auc_scan_workspace_bytes(int64_t rows, int64_t n);
int launch_auc_scan(AucScanArgs a, void* workspace, hipStream_t stream);
// K3c: workspace for the curve passes; count (tile sums + tie-group tails, per-row scan, G_r
// into a.sizes), emit (the compact ascending curves; a.row_off from the host after reading
// sizes) and the sync-free recall-at-fixed-precision chain (count + emit + search + finalize).
int64_t curve_workspace_bytes(int64_t rows, int64_t n, bool rafp);
// K3m: merge two descending-sorted (score, u32 payload) runs into ko / vo (merge path)
// va / vb may be null: the payload is then base_a + i (base_b + j), the sample's position.
// splits: merge_splits_count(na + nb) int64 of scratch.
constexpr int kMergeTile = 2048;
int64_t merge_splits_count(int64_t n);
int launch_merge_desc(const float* ka, const uint32_t* va, int64_t na, uint32_t base_a, const float* kb,
                      const uint32_t* vb, int64_t nb, uint32_t base_b, float* ko, uint32_t* vo, int64_t* splits,
                      hipStream_t stream);
int launch_curve_count(AucScanArgs& a, void* workspace, bool rafp, hipStream_t stream);
int launch_curve_emit(AucScanArgs a, void* workspace, bool rafp, hipStream_t stream);
int launch_rafp(AucScanArgs a, void* workspace, hipStream_t stream);

}  // namespace tea

namespace tea {

// ------------------------------------------------------------------ K4 binned histograms
struct BinnedArgs {
  const void* input = nullptr;  // element (i, j) at i * in_row_stride + j * in_col_stride
  DType in_dt = DType::f32;
  int64_t n = 0;  // samples
  int64_t c = 0;  // classes / labels / tasks
  int64_t in_row_stride = 0;
  int64_t in_col_stride = 0;
  const void* target = nullptr;
  DType tg_dt = DType::i64;
  int mode = 0;  // 0: target(i, j) == 1 is positive; 1: labels, target(i) == j
  int64_t tg_row_stride = 0;
  int64_t tg_col_stride = 0;
  const float* thr = nullptr;  // [T] sorted ascending
  int T = 0;
  int uniform = 0;             // thr is exactly torch.linspace(0, 1, T) (host-known)
  unsigned* ws = nullptr;      // [16 replicas, T + 1, c, 2] u32, zero on entry, left zeroed
  unsigned* slab = nullptr;    // dense path scratch [G, (T + 1) * c] u32, no zero contract
  float* tp = nullptr;         // outputs (accumulated): index k * out_k_stride + j * out_c_stride
  float* fp = nullptr;
  float* fn = nullptr;
  int64_t out_k_stride = 0;
  int64_t out_c_stride = 0;
};
int64_t binned_workspace_words(int T, int64_t c);
int64_t binned_slab_words(int T, int64_t c);  // 0 when the dense path is not used
struct BinnedFinalizeArgs {
  const float* tp = nullptr;  // [T, rows] counts, element (k, r) at k * k_stride + r * r_stride
  const float* fp = nullptr;
  const float* fn = nullptr;  // needed for AUPRC
  int64_t k_stride = 0, r_stride = 0;
  int T = 0;
  int64_t rows = 0;
  double* out_auroc = nullptr;  // [rows] float64 (reference: trapz(...).double())
  float* out_auprc = nullptr;   // [rows] float32
  float* out_prec = nullptr;    // [rows, T + 1] float32 binned PR curve (precision, then 1)
  float* out_rec = nullptr;     // [rows, T + 1] float32 (recall, then 0)
};
int launch_binned_finalize(const BinnedFinalizeArgs& a, hipStream_t stream);
int launch_binned(const BinnedArgs& a, hipStream_t stream);

}  // namespace tea

namespace tea {

// ------------------------------------------------------------------ K5 column moments
struct MomentsArgs {
  const void* x = nullptr;  // element (i, j) at i * x_row_stride + j * x_col_stride
  DType x_dt = DType::f32;
  int64_t x_row_stride = 0, x_col_stride = 0;
  const void* t = nullptr;
  DType t_dt = DType::f32;
  int64_t t_row_stride = 0, t_col_stride = 0;
  const void* w = nullptr;  // optional per-row weight
  DType w_dt = DType::f32;
  int64_t w_stride = 0;
  int64_t n = 0, d = 0;
  float* sse = nullptr;  // [d] outputs (accumulated), element j at j * out_stride
  float* st = nullptr;
  float* stt = nullptr;
  float* sx = nullptr;
  float* sw = nullptr;   // scalar
  int64_t out_stride = 1;
  double* ws = nullptr;  // [ws_blocks, n_requested_stats * d + 1] FP64 partials (caller-allocated)
  int ws_blocks = 0;
  int overwrite = 0;     // 1: outputs are written (=), not accumulated (fresh functional buffers)
  // fused functional compute (post-processing of the column sums inside the finalize):
  //   1 MSE raw_values -> mse_out[d]       2 MSE uniform_average -> mse_out scalar (needs sse, sw)
  //   3 R2 raw_values  -> mse_out[d]       4 R2 uniform_average, 5 R2 variance_weighted -> scalar
  //   (R2 needs sse = RSS, st, stt; num_obs / num_regressors give tss and the adjusted score)
  int mse_mode = 0;
  float* mse_out = nullptr;
  float* mse_part_f = nullptr;  // [2 d] scratch: per-column values (+ tss) for the scalar modes
  int64_t num_obs = 0;
  int num_regressors = 0;
  // one-launch form (f32 x / t with unit column stride, d >= 4, f32 or no weight): per column
  // tile, R row-chunk blocks hand FP64 partials to the tile's last arriver (write-through
  // stores + ticket); the scalar modes add one more ticket over the tiles.
  double* part = nullptr;       // column_moments_v2_ws_doubles(...) doubles
  unsigned* tickets = nullptr;  // [tiles + 1], zero, left zero
  int v2_cg = 0;                // column groups (of 4) per tile: 4 / 16 / 64; 0 = two-launch form
  int v2_r = 0;                 // row chunks per tile
  int64_t v2_chunk = 0;         // rows per chunk
  int v2_pipe = 0;              // two batches of loads in flight per thread (0: one)
  // deferred mode (class updates): each block ADDS its FP64 column partials to its own slot of
  // pend ([slots][ns][d] then [slots] weight totals / row counts) and the launch ends there;
  // launch_moments_fold folds the slots into the float32 states when they are read
  double* pend = nullptr;
  int pend_slots = 0;
  int v2_skip_fold = 0;         // A/B only: stop after the partial stores (results invalid)
};
int column_moments_blocks(int64_t n, int64_t d);
// v2 plan: whether it applies, and its geometry / workspace size (doubles and tickets)
bool column_moments_v2_plan(MomentsArgs& a, int64_t* ws_doubles, int64_t* tickets);
constexpr int kMomentsPendSlots = 64;
// the deferred-mode slot layout: statistic k of the set sits in slot row k, which holds for the
// sets {sse} (need 1), {sse, st, stt} (7) and {sse, st, stt, sx} (15) only: 0 for any other set
// (constexpr: callable from the fold kernel too)
constexpr int moments_ns_of(int need) { return need == 1 ? 1 : need == 7 ? 3 : need == 15 ? 4 : 0; }
constexpr int moments_need(const MomentsArgs& a) {
  return (a.sse ? 1 : 0) | (a.st ? 2 : 0) | (a.stt ? 4 : 0) | (a.sx ? 8 : 0);
}
constexpr int moments_ns(const MomentsArgs& a) { return moments_ns_of(moments_need(a)); }
// pending slots r < rows_used of a deferred-mode pend buffer -> outputs (+= in float32; sse /
// st / stt / sx at out_stride, sw scalar), slots zeroed
int launch_moments_fold(const MomentsArgs& a, int rows_used, hipStream_t stream);
int launch_column_moments(const MomentsArgs& a, hipStream_t stream);

// ------------------------------------------------------------------ K5b per-row weighted sums
// One pass over [rows, n] x (and t, w) producing per row, in FP64, any of
//   WX = sum w x   WT = sum w t   W = sum w   SSE = sum (x - t)^2   WSSE = sum w (x - t)^2
//   WTT = sum w t^2   TMIN / TMAX = min / max t
//   COUNT = n      RANGE = (merged TMAX output) - (merged TMIN output)
// (w: an elementwise weight tensor, or the scalar w_scalar), merged straight into state tensors:
// each output applies op (= / += / min / max) in its own dtype, so a single launch (two for
// long rows) is the whole update of Sum / Mean / PSNR / ClickThroughRate / WeightedCalibration,
// including a windowed metric's ring-slot write and its lifetime accumulation.
enum RowStat : int {
  kWX = 0, kWT = 1, kW = 2, kSSE = 3, kWSSE = 4, kWTT = 5,  // sums
  kTMIN = 6, kTMAX = 7,                                      // extrema
  kCOUNT = 8, kRANGE = 9                                     // derived
};
constexpr int kRowSums = 6, kRowRaw = 8;
enum RowOp : int { kSet = 0, kAdd = 1, kMin = 2, kMax = 3 };
constexpr int kRowSumsMaxOut = 10;
struct RowSumsOut {
  void* p = nullptr;  // element r at r * stride
  DType dt = DType::f64;
  int64_t stride = 0;
  int stat = 0;
  int op = 0;
  int first_row_only = 0;  // a scalar state fed by row 0 only (e.g. a shared count)
};
struct RowSumsArgs {
  const void* x = nullptr;  // element (r, i) at r * x_rs + i * x_cs
  DType x_dt = DType::f32;
  int64_t x_rs = 0, x_cs = 1;
  const void* t = nullptr;
  DType t_dt = DType::f32;
  int64_t t_rs = 0, t_cs = 1;
  const void* w = nullptr;
  DType w_dt = DType::f32;
  int64_t w_rs = 0, w_cs = 1;
  double w_scalar = 1.0;
  int64_t rows = 0, n = 0;
  int need = 0;  // bit mask of the raw stats to reduce (WX .. TMAX)
  int nout = 0;
  RowSumsOut out[kRowSumsMaxOut];
  double* ws = nullptr;  // [rows, blocks, kRowRaw] partials when blocks > 1
  unsigned* ticket = nullptr;  // [rows] zeroed arrival counters: one-launch fold (left zeroed)
  int wt = 0;            // with ticket: write-through partials instead of the fat-block fold
  int blocks = 1;        // blocks per row
  // deferred mode (long rows, ADD outputs of sums / W / COUNT only): every grid block ADDS its
  // FP64 partials - already scaled by a scalar weight, W and COUNT included - to its own slot of
  // pend ([rows][kRowPendStats][pend_blocks]) and the launch ends there; launch_row_sums_fold
  // applies the slots to the outputs when the states are read
  double* pend = nullptr;
  int pend_blocks = 0;
};
// ------------------------------------------------------------------ K4b per-sample binned AUROC
// the reference-default multiclass_binned_auroc (binned_auroc.py:189-215): out[i] = the binned
// AUROC of sample i's true-class score against its other classes (csrc/kernels/binned_auroc.hip)
struct SampleAurocArgs {
  const float* input = nullptr;  // [n, c], unit column stride
  int64_t n = 0, c = 0, row_stride = 0;
  const void* target = nullptr;  // [n] int64 / int32
  DType tg_dt = DType::i64;
  int64_t tg_stride = 1;
  const float* thr = nullptr;  // [T] ascending
  int T = 0;
  float* out = nullptr;  // [n]
  int* err = nullptr;    // bit 0: a label outside [0, c)
};
int launch_sample_binned_auroc(const SampleAurocArgs& a, hipStream_t stream);

constexpr int kRowPendStats = kRowSums + 3;  // the six sums, COUNT, then the target min / max
                                             // (a slot's extrema are valid while its COUNT != 0)
constexpr int kRowPendBlocks = 2048;
// pending slots b < blocks_used of every row -> the outputs of a (ADD), slots zeroed
int launch_row_sums_fold(const RowSumsArgs& a, int blocks_used, hipStream_t stream);
int row_sums_blocks(int64_t rows, int64_t n);       // two-launch grid (partials + combine)
int row_sums_fold_blocks(int64_t rows, int64_t n);
int row_sums_wt_blocks(int64_t rows, int64_t n);  // one-launch fold (needs a ticket)
int launch_row_sums(const RowSumsArgs& a, hipStream_t stream);
// the same update on host memory (CPU tensors): the small-batch twin of the kernel
void row_sums_host(const RowSumsArgs& a);

// ------------------------------------------------------------------ K6 normalized entropy
struct NeArgs {
  const void* x = nullptr;
  DType x_dt = DType::f32;
  int64_t x_row_stride = 0;
  const void* t = nullptr;
  DType t_dt = DType::f32;
  int64_t t_row_stride = 0;
  const void* w = nullptr;
  DType w_dt = DType::f32;
  int64_t w_row_stride = 0;
  int64_t rows = 0, n = 0;
  int from_logits = 0;
  double* out = nullptr;  // [rows, 3]: sum w*bce, sum w*t, sum w (accumulated)
  int* err = nullptr;
  // optional: order-preserving u64 keys of max(x) and (complemented) min(x) over the launch,
  // atomicMax-accumulated (zero = unset), so a deferred range error can print the batch range
  unsigned long long* range = nullptr;
  double* ordered_ws = nullptr;  // deterministic mode: [rows * 3, ne_sums_blocks] partials
};
int ne_sums_blocks(int64_t n);
int launch_ne_sums(const NeArgs& a, hipStream_t stream);

// deterministic fold: out[v] += sum_{p < parts} ws[v * parts + p], summed in index order
int launch_ordered_sum(const double* ws, int64_t nvals, int64_t parts, double* out, hipStream_t stream);

}  // namespace tea

namespace tea {

// ------------------------------------------------------------------ K7 perplexity
struct PerplexityArgs {
  const void* input = nullptr;  // [rows, v] logits (row stride)
  DType in_dt = DType::f32;
  int64_t rows = 0, v = 0, row_stride = 0;
  const void* target = nullptr;  // [rows] (stride)
  DType tg_dt = DType::i64;
  int64_t tg_stride = 1;
  int has_ignore = 0;
  int64_t ignore_index = 0;
  double* out = nullptr;  // [2]: sum of -log p(target), token count (accumulated)
  int* err = nullptr;
  double* ordered_ws = nullptr;  // deterministic mode: [2, perplexity_blocks] partials
};
int perplexity_blocks(const PerplexityArgs& a);  // grid of the launch launch_perplexity makes
int launch_perplexity(const PerplexityArgs& a, hipStream_t stream);

}  // namespace tea

namespace tea {

// ------------------------------------------------------------------ K8 FID covariance
struct FidCovArgs {
  const float* act = nullptr;  // [n, ld] activations (row stride, unit column stride)
  int64_t n = 0, d = 0, row_stride = 0;
  int64_t ld = 0;               // loaded width: d rounded up to 4 (columns [d, ld) must be 0)
  const float* zeros = nullptr;  // >= 16 B of zeros (the source of masked LDS-DMA slots)
  float* cov = nullptr;     // [d, d] contiguous, += act^T act
  float* colsum = nullptr;  // [d], += column sums (optional)
  int split = 1;            // K-range items per output tile (> 1: partials + fix-up pass)
  float* ws = nullptr;      // split > 1: fid_cov_workspace_bytes(d, split) of scratch
};
// split-K factor the launcher would pick for [n, d] on this device (env TORCHEVAL_AMD_K8_SPLIT
// overrides) and the scratch it needs
int fid_cov_split(int64_t n, int64_t d);
// K8 product path: 2 = bf16 MFMA on the exact three-way split, staged once per block (default);
// 1 = the same split done per wave (TORCHEVAL_AMD_K8_MODE=1); 0 = FP32 MFMA (TORCHEVAL_AMD_K8_EXACT=1)
int fid_cov_mode();
int64_t fid_cov_workspace_bytes(int64_t d, int split);
int launch_fid_cov(const FidCovArgs& a, hipStream_t stream);

}  // namespace tea

// ------------------------------------------------------------------ K2 multilabel accuracy
namespace tea {
struct MultilabelArgs {
  const void* x = nullptr;  // [n, c] scores (f32 / bf16 / f16), rows at x_row_stride
  DType x_dt = DType::f32;
  int64_t x_row_stride = 0;
  const void* t = nullptr;  // [n, c] targets (f32 / i64 / i32 / u8 / bool)
  DType t_dt = DType::f32;
  int64_t t_row_stride = 0;
  int64_t n = 0, c = 0;
  float threshold = 0.5f;
  int k = 0;         // > 0: top-k labels instead of thresholding
  int criteria = 0;  // 0 exact_match, 1 hamming, 2 overlap, 3 contain, 4 belong
  float* num_correct = nullptr;  // accumulated
  float* num_total = nullptr;    // optional: += total (block 0)
  double total = 0.0;
  unsigned long long* fold_ws = nullptr;
};
int multilabel_max_topk_cols();
int launch_multilabel(const MultilabelArgs& a, hipStream_t stream);
}  // namespace tea

// ------------------------------------------------------------------ K3a radix sort
namespace tea {
struct RadixArgs {
  const float* in = nullptr;  // [rows, n] scores, rows at in_row_stride (unit column stride)
  int64_t in_row_stride = 0;
  int64_t rows = 0, n = 0;
  int64_t tiles = 0;          // radix_sort_tiles(rows, n)
  uint32_t* keys0 = nullptr;  // ping-pong [rows * n]
  uint32_t* vals0 = nullptr;
  uint32_t* keys1 = nullptr;
  uint32_t* vals1 = nullptr;
  uint32_t* hist = nullptr;   // [rows, tiles, 256] per-tile digit counts of the current pass
  uint32_t* groups = nullptr; // 4 pass regions (`region` cells apart) of [rows, ngroups, 256] digit
                              // counts per group of tiles.  Self-cleaning: passes 1-3 clear the
                              // previous pass's region; pass 3's is cleared by the next sort's pass 0
                              // (a last-block-done clear in the final downsweep serialised 512
                              // same-address atomics: +5 us per 1M-key sort)
  int64_t region = 0;
  uint32_t* dirty = nullptr;  // cells of region 3 left to clear (written by the final downsweep)
  int64_t ngroups = 0;        // radix_sort_groups(tiles)
  float* out_sorted = nullptr;  // [rows, n] descending
  int32_t* out_order = nullptr; // [rows, n] source index within the row (or the payload)
  // optional payload carried instead of the source index (pass 0 reads it, coalesced):
  //   1: f32 bits of payload[row * payload_row_stride + i]  (binary targets)
  //   2: int32 of payload[row * payload_row_stride + i]     (class labels; row stride 0 = shared)
  int payload_kind = 0;
  const void* payload = nullptr;
  DType payload_dt = DType::f32;
  int64_t payload_row_stride = 0;
  // onesweep mode (radix_onesweep_ok): one histogram launch for all four digits, then four
  // passes that each rank, look back and scatter in ONE launch (no upsweeps).  Self-cleaning,
  // zero-initialised workspaces:
  uint32_t* os_hdr = nullptr;     // [16]: [4..7] dirty extents of the status / group planes,
                                  // [8] look-back timeout flag (cleared by each sort's histogram
                                  // launch, so it describes the latest onesweep sort of the stream)
  uint32_t* os_watch = nullptr;   // host (pinned) word: the histogram launch copies [8] there before
                                  // clearing it, so the host learns of a timed-out sort one sort
                                  // later without a device-to-host copy on the stream
  int spin_limit = 1 << 22;       // look-back polls before a tile gives up (TORCHEVAL_AMD_K3_SPIN_LIMIT)
  uint32_t* os_g = nullptr;       // [rows, 8 copies, 4, 256] digit totals (hist kernel; cleared by pass 3)
  uint32_t* os_status = nullptr;  // 2 planes of [rows * tiles, 256] ready-flagged tile counts
  int64_t os_splane = 0;          // words per status plane
  unsigned long long* os_gacc = nullptr;  // 2 planes of [rows * ngroups, 256] (arrivals << 32 | sum)
  int64_t os_gplane = 0;          // words per group plane
  // optional K3 tile-sum fold (onesweep, payload kinds 1 / 2): the last pass adds each
  // 1024-sample output tile's (sum a, sum b) of the sorted payload (a = t, b = 1 - t; kind 2:
  // t = [label == row]) into fold_ab, which pass 0 zeroes; auc_scan then skips tile_sums
  double* fold_ab = nullptr;      // [rows, fold_otiles, 2]
  int64_t fold_otiles = 0;        // ceil(n / 1024)
  int fold_probe = 0;             // A/B probe (TORCHEVAL_AMD_K3_FOLD_PROBE): 1 no atomics, 2 no fold work
  // 0: descending (NaN first); ~0u: ascending (NaN last, as torch.sort ascending), both stable -
  // XORed into every key at load and out of it at the final store
  uint32_t key_xor = 0;
  // splitter-bucket mode (radix_bucket_ok; onesweep workspaces required): 255 equal-frequency
  // splitters per row from a sorted sample, ONE stable onesweep pass scatters the keys into the
  // 256 buckets they delimit, and one workgroup per bucket finishes it in LDS
  uint32_t* bkt_spl = nullptr;  // [rows, 256] splitters (sample kernel)
  uint32_t* bkt_cnt = nullptr;  // [rows, 256] bucket sizes (the pass's first tile)
};
bool radix_bucket_ok(int64_t rows, int64_t n);    // the rows / lengths the bucket mode takes
bool radix_onesweep_ok(int64_t rows, int64_t n);  // the tiling the onesweep passes take
int64_t radix_onesweep_status_words(int64_t rows, int64_t n);
int64_t radix_onesweep_group_words(int64_t rows, int64_t n);
int radix_sort_rounds(int64_t rows, int64_t n);  // keys per thread of the tiling
int64_t radix_sort_tiles(int64_t rows, int64_t n);
int64_t radix_sort_groups(int64_t tiles);
int launch_transpose_f32(const float* in, int64_t n, int64_t c, int64_t ld_in, float* out, hipStream_t stream);
int launch_radix_sort_desc(const RadixArgs& a, hipStream_t stream);
// ------------------------------------------------------------------ K10b retrieval top-k
struct RetrievalArgs {
  const float* x = nullptr;        // [n] scores
  const float* t = nullptr;        // [n] targets
  const int64_t* q = nullptr;      // [n] query ids (null: every sample is query 0)
  int64_t n = 0, Q = 0;
  int k = 0;                        // 1..64
  float* topk = nullptr;            // [Q, k] state (best first, -inf padded)
  float* target_state = nullptr;    // [Q, k]
  int64_t* count = nullptr;         // [Q] valid entries (<= k)
  int* counts = nullptr;            // [Q] zeroed scratch (left zeroed)
  int* offsets = nullptr;           // [Q + 1] scratch
  int* cursor = nullptr;            // [Q] scratch
  uint32_t* rec_key = nullptr;      // [n] scratch
  uint32_t* rec_idx = nullptr;      // [n] scratch
};
constexpr int kRetrievalMaxLds = 64 * 1024;  // 2 x Q int32 of LDS: Q <= 8192
int launch_retrieval_topk(const RetrievalArgs& a, hipStream_t stream);

}  // namespace tea

namespace tea {

// ------------------------------------------------------------------ K9b symmetric eigenvalues
struct SymEigArgs {
  const double* a = nullptr;  // [n, n] symmetric, contiguous
  int64_t n = 0;
  int64_t ld = 0;             // slot stride, symeig_slot_stride(n)
  double* d = nullptr;        // [n] tridiagonal diagonal (workspace)
  double* e = nullptr;        // [n] off-diagonal (workspace)
  double* lam = nullptr;      // [n] eigenvalues, ascending
  unsigned long long* slots = nullptr;  // 2 planes of [n - 2, ld] hand-off slots,
                                        // symeig_slot_bytes(n) (sentinel-filled by the launcher)
  unsigned* ctl = nullptr;    // 128 B: ctl[1] abort word (zeroed by the launcher)
  int* grid = nullptr;        // symeig_grid_bytes(): Sturm counts of the eigenvalue search grid
  double* tail = nullptr;     // symeig_tail_bytes(): the trailing block the one-workgroup tail finishes
};
// 0 when the on-chip one-launch reduction fits this device (grid / rows per block out)
int symeig_plan(int64_t n, int* grid, int* rows_per_block);
int64_t symeig_slot_stride(int64_t n);
int64_t symeig_slot_bytes(int64_t n);
int64_t symeig_grid_bytes();
int64_t symeig_tail_bytes();
// 0 launched, 1 unsupported size, 2 HIP error, 3 cooperative launch refused
int launch_symeig(const SymEigArgs& a, hipStream_t stream);

}  // namespace tea

namespace tea {
// K9c: factor the b x b diagonal block A[k0:k0+b, k0:k0+b] (row-major, leading dimension lda)
// in place into its lower Cholesky factor (upper part zeroed) and write its inverse to Linv
// [b, b]; a non-positive pivot sets *info = k0 + column + 1 (if still 0).  b <= 64.
int potrf_block_size();
// K9d (cholesky.hip): the whole blocked Cholesky in one persistent launch.  L: padded
// [64 nt, 64 nt] factor, Linv: nt x 64 x 64, ctl: 1 int (ticket), status: 2 ints (info, abort)
int cholesky_tiles(int64_t n);
// fid_prep.hip: S = ((C + C^T) / 2 - n mu mu^T) / (n - 1) in FP64 from the FP32 K8 states;
// M[i][j] = M[j][i] above the diagonal (in place)
// trapz.hip: per-row trapezoid area of x-sorted rows (x, y f32 [rows, n]) -> out f32 [rows];
// part: FP64 scratch of rows * trapz_blocks(n)
int trapz_blocks(int64_t n);
int launch_trapz_sorted(const float* x, const float* y, int64_t rows, int64_t n, double* part, float* out,
                        hipStream_t stream);
int launch_cov_finalize(const float* C, const float* colsum, double n, int64_t d, double* S, hipStream_t stream);
int launch_sym_fill_upper(double* M, int64_t ld, int64_t n, hipStream_t stream);
int launch_fid_finish(const float* sum1, double n1, const float* sum2, double n2, int64_t d, const double* s1,
                      int64_t ld1, const double* s2, int64_t ld2, const double* lam, int64_t r, float* out,
                      hipStream_t stream);
int launch_cholesky(const double* A, int64_t lda, int64_t n, double* L, double* Linv, int* ctl, int* status,
                    hipStream_t stream, unsigned long long* trace = nullptr);
int launch_potrf_block(double* A, int64_t lda, int k0, int b, double* Linv, int* info, hipStream_t stream);
// K9p (pivchol.hip): pivoted FP64 Cholesky, one cooperative launch.  slots: pivchol_slot_words(n)
// 64-bit words, w: [N, N] doubles, N = pivchol_padded(n); info {rank, status}; ctl 1 word.
// 0 launched, 3 not co-schedulable, 4 n unsupported
int pivchol_padded(int64_t n);
int64_t pivchol_slot_words(int64_t n);
int launch_pivchol(const double* A, int64_t lda, int64_t n, unsigned long long* slots, double* w, int* piv, int* info,
                   unsigned* ctl, hipStream_t stream, unsigned long long* trace = nullptr);
}  // namespace tea

namespace tea {
// C3: reduce a gathered [ws][row_bytes] metric-state buffer segment by segment across ranks
// (rank 0 first) into ``out`` (same byte layout).  op: 0 sum, 1 max, 2 min; dtype: DType.
constexpr int kSegMax = 32;
struct SegReduceArgs {
  const uint8_t* rows = nullptr;
  uint8_t* out = nullptr;
  int ws = 1;
  int64_t row_bytes = 0;
  int nseg = 0;
  int64_t off[kSegMax] = {};        // byte offset of each segment in a row
  int64_t first[kSegMax + 1] = {};  // prefix sum of segment element counts
  int dtype[kSegMax] = {};
  int op[kSegMax] = {};
};
int launch_seg_reduce(const SegReduceArgs& a, hipStream_t stream);
// copy ``bytes`` (multiple of 16) of src to dst and append this rank's flag words as f32 (hi16,
// lo16) pairs in slot ``rank`` of a zeroed [ws][words][2] block (err null: zeros)
int launch_snapshot_flags(const void* src, void* dst, int64_t bytes, const int* err, int words, int rank, int ws,
                          hipStream_t stream);
// summed [ws][words][2] slots -> int32 [words], max over ranks
int launch_merge_flag_slots(const float* slots, int* out, int words, int ws, hipStream_t stream);
// test support (csrc/kernels/testing.hip): one lane spins until *flag != 0 or max_ms elapse
// low-latency host read (hostread.hip): words <= kHostReadWords int32 from src into a pinned,
// device-mapped host slot [seq, words...], published by a system-scope release store of seq
constexpr int kHostReadWords = 14;
int launch_publish_words(const int32_t* src, int words, int32_t* slot_dev, int32_t seq, hipStream_t stream,
                         const int32_t* src2 = nullptr, int words2 = 0);
int launch_spin_on_flag(const int* flag, int64_t max_ms, hipStream_t stream);
}  // namespace tea
