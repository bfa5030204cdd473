// Host-side launch interface of the gfx950 kernels (internal to libclipembed).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ce {

typedef uint16_t bf16_t;

enum Act { ACT_NONE_ = 0, ACT_GELU_ = 1, ACT_QGELU_ = 2 };

// out[map_o(m)][n] = act(sum_k A[m][k] * W[n][k] + bias[n]) + resid[map_r(m)][n]
//   A [M][K] bf16 (row stride lda), W [N][K] bf16 (nn.Linear layout, row stride ldw).
//   map_x(m) = (m / grp) * x_gs + x_go + (m % grp); grp == 0 means the identity map.
// Requirements (checked by the launcher): K % 64 == 0, N % 64 == 0, 16-B aligned rows.
struct GemmParams {
    const bf16_t* A; long lda;
    const bf16_t* W; long ldw;
    int M, N, K;
    const float* bias;                 // nullable, [N]
    const float* resid; long ldr;      // nullable, f32
    void* out; long ldo;               // f32 or bf16
    int grp, o_gs, o_go, r_gs, r_go;
    int gm = 0;                        // tile-order M-group (set by launch_gemm)
    // split-K tail (set by launch_gemm): the last `tail` tiles are computed as `split` K-chunks each
    // (partial f32 tiles into `part`), summed in fixed order by a fixup kernel
    float* part = nullptr; long part_elems = 0;
    int tail = 0, split = 1;
    int tail_only = 0;                     // 4-phase kernel: run only the split-K chunks (SCHED 11's tail)
    // LayerNorm folded into the GEMMs around it (EPI_LN_STATS / EPI_LN_FOLD):
    //   producer (residual GEMM, f32 out): also xb[m][n] = bf16(out) and, per 64-column slab,
    //     stats_part[m][n/64] = (mean, sum of squared deviations) of the outputs
    //   consumer: A = bf16(x) (un-normalised), W = bf16(gamma o W); out = act(rstd_m * (acc -
    //     mu_m * fold_c[n]) + bias[n]) with fold_stats[m] = (mu, rstd) and bias = b + W beta
    bf16_t* xb = nullptr;
    float2* stats_part = nullptr;
    const float2* fold_stats = nullptr;
    const float* fold_c = nullptr;
    // residual stream as two bf16 planes (EPI_LN_STATS_HL / EPI_HL_F32): residual = rhl[m][n] +
    // rhl[hl_plane + m][n] (row stride ldr); EPI_LN_STATS_HL writes its output the same way into
    // xb / xb + hl_plane (row stride ldo) instead of out f32 + the bf16 copy
    const bf16_t* rhl = nullptr;
    long hl_plane = 0;
    // de-synchronisation of the first round of workgroups (set by launch_gemm): blocks b in
    // [stagger_lo, stagger_hi) with bit `stagger_bit` of b set (stagger_bit < 0: all of them) sleep
    // `stagger` x 127 x 64 cycles before starting, so that later rounds keep half the CUs in their
    // epilogue while the other half run MFMAs instead of the whole chip alternating between the two
    int stagger = 0, stagger_lo = 0, stagger_hi = 0, stagger_bit = -1;
    unsigned long long* trace = nullptr;   // diagnostic timeline, [block][4] (set_gemm_trace)
    int trace_n = 0;
    int variant = 0;                       // kernel-variant bits for A/B (set_gemm_variant)
    // the caller's request for one tile per four-wave workgroup (grid = tiles): small grids that
    // run beside another stream's persistent GEMMs (the text tower beside the image tower) take
    // CUs one tile at a time as they free up (GEMM_VAR_SMALL_ONETILE, default on)
    int onetile = 0;
    // packed rows (the text tower's pooled-only calls): only the first *m_dev of the M rows are live;
    // tiles past them exit.  Implies one tile per workgroup and no split-K tail (launch_gemm).
    const int* m_dev = nullptr;
    // bf16 output with an activation (EPI_PLAIN, no residual): also store the pre-activation values
    // (bias added) here, same layout as out (the training forward keeps both for the backward)
    bf16_t* pre_out = nullptr;
    // activation-backward epilogue (launch_gemm_act_bwd only): out = bf16(bf16(acc) * act'(bwd_pre))
    // with bwd_pre the forward's pre-activation copy (same layout as out), and per 128-row block of
    // the output the column sums of out into bwd_part[m / 128][n]
    const bf16_t* bwd_pre = nullptr;
    float* bwd_part = nullptr;
    // the process-wide schedule knobs (knobs.h), read once by launch_gemm so one launch never mixes
    // values another thread sets meanwhile
    // (snap: set by the snapshot, so launch_gemm_act_bwd acts on gemm_act_bwd_fused's decision)
    struct {
        int sched = 1, autom = 1, splitk = 1, groupm = 4, stagger = 0, snap = 0;
    } kn;
};
// EPI_LN_STATS_HL: EPI_LN_STATS with the residual stream as hi/lo bf16 planes in and out;
// EPI_HL_F32: residual from hi/lo planes, plain f32 output (the tower's last residual GEMM)
enum GemmEpi { EPI_PLAIN = 0, EPI_LN_STATS = 1, EPI_LN_FOLD = 2, EPI_LN_STATS_HL = 3, EPI_HL_F32 = 4 };
hipError_t launch_gemm(const GemmParams& p, int act, bool out_bf16, hipStream_t s, int epi = EPI_PLAIN);
// dX GEMM of the MLP's c_proj in the text-tower backward with the activation backward and the c_fc
// bias column sums in its epilogue (GemmParams::bwd_pre / bwd_part; act = the forward activation,
// ACT_GELU or ACT_QGELU): the four-wave persistent kernel on the default policy, bf16 out, no bias /
// residual, N % 128 == 0, out and bwd_pre of row stride N.  gemm_act_bwd_fused takes the knob
// snapshot into p and says whether a launch of that p takes the fused path; launch_gemm_act_bwd(p)
// then decides on the same snapshot (hipErrorNotSupported if not fused: the caller runs launch_gemm +
// launch_act_bwd_colsum).  bwd_part holds (M + 127) / 128 rows of N floats.
bool gemm_act_bwd_fused(GemmParams& p, int act);
hipError_t launch_gemm_act_bwd(const GemmParams& p, int act, hipStream_t s);
// (mu, rstd) per row from the 64-column slab statistics of an EPI_LN_STATS launch (Chan's
// combination; eps 1e-5): stats[r] from part[r][0 .. nslab-1]
// (m_dev: packed rows, only the first *m_dev of the `rows` are live)
hipError_t launch_ln_stats_finalize(float2* stats, const float2* part, int rows, int nslab, hipStream_t s,
                                    const int* m_dev = nullptr);
int set_gemm_schedule(int v);   // returns previous
int current_gemm_sched();       // the current main-loop schedule (1 = default)
int set_gemm_splitk(int on);     // split-K tail on/off (default on); returns previous
int set_gemm_variant(int bits);  // kernel-variant bits for A/B (GEMM_VAR_*); returns previous
int set_gemm_auto(int mode);     // shape policy (CE_GEMM_AUTO: 0 off, 1 default, 2 / 3 wider SCHED 11); returns previous
// launch counters per kernel path; index = path base + epilogue (EPI_PLAIN/LN_STATS/LN_FOLD)
enum GemmPath { GEMM_PATH_W4PP = 0, GEMM_PATH_NT = 3, GEMM_PATH_FIXUP = 6, GEMM_PATH_OTHER = 9, GEMM_PATH_W2 = 10,
                GEMM_PATH_COUNT = 13 };
void gemm_path_counts(long long* out, int n, bool reset);
void set_gemm_trace(unsigned long long* buf, long n);   // diagnostics: per-block timeline of the next launches
float* gemm_kernel_api_workspace(long* elems);   // per-device partial-tile buffer (kernel-level API)
constexpr long kGemmPartElems = 256L * 256 * 256;   // partial-tile workspace a handle provides (64 MB)

// Weight-gradient GEMM with MN-major operands (gemm_tn.hip): C[m][n] = scale_m * sum_k A[k][m] B[k][n]
//   A [K][lda], B [K][ldb] bf16 (row-major activations, reduction down their rows), C [M][ldc] f32;
//   scale_m = scale for m < scale_rows else 1.  M % 256 == 0, N % 256 == 0, 16-B aligned rows.
//   part (nullable, part_elems floats): split-K partial tiles; null = one workgroup per tile.
struct TnParams {
    const bf16_t* A; long lda;
    const bf16_t* B; long ldb;
    int M, N, K;
    float* C; long ldc;
    float* part = nullptr; long part_elems = 0;
    int split = 1;                       // set by the launcher
    int scale_rows = 0; float scale = 1.f;
};
hipError_t launch_gemm_tn(const TnParams& p, hipStream_t s);
int gemm_tn_split(int M, int N, int K, long part_elems);   // the K-split launch_gemm_tn picks (0: bad shape)

// Multi-head attention over a packed QKV activation.
//   qkv [B*L][3*D] bf16 (q | k | v, head h at columns h*64 .. h*64+63 of each part)
//   out [B*L][D]   bf16 (heads concatenated), softmax(q k^T / sqrt(64) [+ causal]) v
// q_prescaled: the q third of qkv already carries kAttnQScale (engine in_proj weights); else the
// kernel scales its Q fragments.
constexpr float kAttnQScale = 0.125f * 1.4426950408889634f;   // log2(e) / sqrt(64)
int set_attn_variant(int var);   // attention forward variant for A/B (381 default, 125; include/clipembed.h); returns previous
int set_fgemm_variant(int v);   // 1 = register-blocked f32 GEMM (default), 0 = the 64 x 64 kernel
hipError_t launch_attention(const bf16_t* qkv, bf16_t* out, int B, int L, int H, bool causal, bool q_prescaled,
                            hipStream_t s, float* lse = nullptr,   // lse: [B][H][L] log2 log-sum-exp (training)
                            const int* seg = nullptr);  // seg: packed sequences (launch_text_pack), L = max length
// The same attention for ONE query row per sequence (row qrows[b], absolute; null: row b*L), keys
// of sequence b only (0..qrows[b]-b*L with causal); out [B][D] bf16 compact.  q pre-scaled as
// launch_attention(q_prescaled).  src/dst (optional): copy the selected rows of the hi/lo planes
// (plane strides splane / dplane elements) to compact rows b of dst.
hipError_t launch_attention_rows(const bf16_t* qkv, const int* qrows, bf16_t* out, int B, int L, int H, bool causal,
                                 const bf16_t* src, long splane, bf16_t* dst, long dplane, hipStream_t s,
                                 const int* seg = nullptr,    // seg: packed causal sequences (row0 = seg[b])
                                 // wq: compute the pooled rows' q here (LN-folded in_proj rows 0..D-1 [D][D],
                                 // fold column sums cq, bias dq, row stats; x = src hi plane); qkv then
                                 // needs only its K and V thirds
                                 const bf16_t* wq = nullptr, const float* cq = nullptr, const float* dq = nullptr,
                                 const float2* stats = nullptr);

// LayerNorm over rows of width D (eps 1e-5, affine), f32 in, f32 or bf16 out.
//   in row  = (r / grp) * i_gs + i_go + r % grp   (grp == 0: identity)
//   out row = (r / grp) * o_gs + o_go + r % grp
struct LNParams {
    const float* in; long ldi;
    void* out; long ldo;
    const float* w; const float* b;
    int rows, D;
    int grp, i_gs, i_go, o_gs, o_go;
    // optional second LayerNorm applied to the first one's output (PACL head LN), with an
    // optional de-interleaving RoPE between the two (pacl.py:147-181; cos/sin [P][D/2]).
    const float* w2; const float* b2;
    const float* rope_cos; const float* rope_sin; int rope_P;
    // optional (f32-output single LN, e.g. ln_pre): bf16 copy of the output and its row (mu, rstd)
    // for an EPI_LN_FOLD consumer
    bf16_t* xb = nullptr;
    float2* stats = nullptr;
    bf16_t* xlo = nullptr;      // with xb: the lo plane of the hi/lo residual stream (xb = hi)
};
hipError_t launch_layernorm(const LNParams& p, bool out_bf16, hipStream_t s);

// Patchify: pixels [B,3,S,S] (f32 or bf16) -> cols [B*G*G][Kp] bf16, col = c*p*p + ky*p + kx,
// zero padded up to Kp.
hipError_t launch_im2col(const void* pix, bool pix_bf16, bf16_t* cols, int B, int S, int patch,
                         int Kp, hipStream_t s);
// x[b*Lv][:] = class_emb + pos[0]  (row 0 of every image)
hipError_t launch_cls_rows(float* x, const float* cls, const float* pos, int B, int Lv, int D,
                           hipStream_t s);
// x[b*ctx+t][:] = tok[ids[b,t]] + pos[t]
hipError_t launch_text_embed(float* x, const int64_t* ids, const float* tok, const float* pos,
                             int B, int ctx, int D, int vocab, hipStream_t s);
// the LN-folded text tower's entry state: x = tok[ids] + pos (f32), hi/lo bf16 planes (xlo may be
// null: xb = bf16(x)), row (mu, rstd).  D in {256, 512, 768, 1024, 1280}.
hipError_t launch_text_embed_stats(float* x, bf16_t* xb, bf16_t* xlo, float2* stats, const int64_t* ids,
                                   const float* tok, const float* pos, int B, int ctx, int D, int vocab,
                                   hipStream_t s, const int* seg = nullptr);   // seg: packed rows (launch_text_pack)
// packed text rows of a pooled-only call: caption b's tokens 0..EOT at rows seg[b]..seg[b+1]-1,
// seg[B] = live rows, sel[b] = seg[b] + EOT position (one workgroup)
hipError_t launch_text_pack(int* sel, int* seg, const int64_t* ids, int B, int ctx, hipStream_t s);
// rows[b] = b*ctx + argmax_t ids[b,t]  (first maximal id; EOT is the largest id)
hipError_t launch_argmax_rows(int* rows, const int64_t* ids, int B, int ctx, hipStream_t s);
// LayerNorm of gathered rows: out[i] = LN(x + rows[i]*row_stride) (f32); rows == nullptr -> rows[i] = i
hipError_t launch_ln_gather(float* out, const float* x, const int* rows, long row_stride, int n,
                            int D, const float* w, const float* b, hipStream_t s);
// Batched f32 GEMM (VALU, 64x64 tiles): C[z][i][j] = alpha * sum_k A[z][i][k] * B'[z] + bias[j]
//   b_nk: B stored [N][K] (C = A B^T) else [K][N] (C = A B).
struct FGemmParams {
    const float* A; long lda, sA;
    const float* B; long ldb, sB;
    float* C; long ldc, sC;
    int M, N, K, batch;
    float alpha;
    const float* bias;     // nullable [N]
    float* Ct; long ldct;  // nullable: also write C^T (batch 1 only)
    int accumulate = 0;    // C += alpha A B' (+ bias) instead of C = ...
};
hipError_t launch_fgemm(const FGemmParams& p, bool b_nk, hipStream_t s);
// rows of D: x / max(||x||, 1e-12)
hipError_t launch_l2norm(float* out, const float* x, int rows, int D, hipStream_t s);
// cross entropy: accum[2] (zeroed by the caller) collects sum/count, finish writes the mean
hipError_t launch_cross_entropy_rows(float* accum, const float* logits, int R, int C,
                                     const int64_t* labels, hipStream_t s);
hipError_t launch_cross_entropy_finish(float* loss, const float* accum, hipStream_t s);
// part: f32 scratch of pacl_pool_part_bytes(max(Bi, Bt), P, D) bytes (per-split partial rows)
hipError_t launch_pacl_pool(const void* vp, bool vp_bf16, int Bi, int P, const float* tp, int Bt,
                            int D, int weight_mode, const float* rope_cos, const float* rope_sin,
                            float* out_img, float* out_txt, float* part, hipStream_t s);
size_t pacl_pool_part_bytes(int R, int P, int D);
// SPARC row step in place on sim [rows][P]: min-max normalise, zero below sigma, divide by sum
hipError_t launch_sparc_weights(float* sim, long rows, int P, float sigma, hipStream_t s);
hipError_t launch_rope(float* out, const float* x, int B, int P, int D, const float* cos_t,
                       const float* sin_t, hipStream_t s);
hipError_t launch_f32_to_bf16(bf16_t* out, const float* in, long n, hipStream_t s);

// ---- SPARC head training (sparc_train.hip) ----
// LayerNorm (eps 1e-5) + Dropout(p) per row of D (% 256, <= 1024): out bf16 or f32, stats[r] = (mu, rstd);
// the keep mask is a counter hash of (seed, (roff + r) * D + c) (roff: the global row of local row 0),
// recomputed by launch_ln_grad
hipError_t launch_ln_drop(const float* x, const float* w, const float* b, long R, int D, float p, uint64_t seed,
                          long roff, void* out, bool out_bf16, float2* stats, hipStream_t s);
// dw, db (overwritten) = the LayerNorm weight / bias gradients through that dropout; scratch >= ln_grad_scratch_floats
long ln_grad_scratch_floats(long R, int D);
hipError_t launch_ln_grad(const float* dy, const float* x, const float2* stats, long R, int D, float p, uint64_t seed,
                          long roff, float* dw, float* db, float* scratch, hipStream_t s);
// io: d loss / d W in, d loss / d S out, per row of P (sparc weights backward, S = raw similarity)
hipError_t launch_align_bwd(const float* S, float* io, long rows, int P, float sigma, hipStream_t s);
// SparcLoss local-term gradient per sample: dR, dR^T [B][T][T] and part[B][3] from R = scale Gn Ln^T (T <= 80)
hipError_t launch_local_grad(const float* R, const float* mask, int B, int T, float w, float* dR, float* dRT,
                             float* part, hipStream_t s);
// g = w (softmax(z) - onehot(row)), loss[row] = lse - z[row]
hipError_t launch_ce_diag_grad(const float* z, int R, int C, float w, float* g, float* loss, hipStream_t s);
// out[z][c][r] = in[z][r][c] (+ add[z][c][r])
hipError_t launch_transpose_add(const float* in, const float* add, float* out, int batch, int R, int C, hipStream_t s);
// x[b][p][d] += scale * v[b][d]
hipError_t launch_bcast_add_mid(float* x, const float* v, int B, int P, int D, float scale, hipStream_t s);

// SparcLoss pieces (pacl.py:516-584)
hipError_t launch_mean_mid(float* out, const float* x, int B, int P, int D, hipStream_t s);   // mean over dim 1
// per-row CE vs labels arange + off
hipError_t launch_ce_diag_rows(float* loss, const float* L, int R, int C, int off, hipStream_t s);
hipError_t launch_sparc_local(float* part, const float* S, const float* mask, int B, int T, hipStream_t s);
// parts[5] = {sum lr, sum lc, sum part[.][0], sum part[.][1], sum part[.][2]} of one shard
hipError_t launch_loss_parts(float* parts, const float* lr, const float* lc, int R, const float* part, int B,
                             hipStream_t s);
// out = wg (P0 + P1) / (2 N) + wl (P2 + P3) / (2 P4)   (wl == 0: no local term)
hipError_t launch_loss_combine(float* out, const float* parts, int N, float global_weight, float local_weight,
                               hipStream_t s);

// Device image preprocessing (preprocess.hip).  Per image: source offset/size, the source rows
// the vertical taps touch [ybase, ybase + nrows), the intermediate's offset, and tap tables:
// bounds (start, count) pairs at bx_off (S output columns, absolute source x) and by_off (S output
// rows, relative to ybase); taps (int32 Pillow fixed point, or f32) at kx_off / ky_off with row
// strides ksx / ksy.
struct PrepMeta {
    long long in_off;
    int H, W;
    int ybase, nrows;
    long long tmp_off;
    int bx_off, by_off;
    int kx_off, ksx, ky_off, ksy;
};
hipError_t launch_preprocess(const uint8_t* images, const PrepMeta* meta, const int* bounds, const void* taps,
                             void* tmp, int B, int max_rows, int S, bool pacl, bool out_bf16, const float* mean,
                             const float* stdv, void* out, hipStream_t s);


// ---- text-tower training (train.hip) ----
// out[c][r] (row stride ldo) = in[r][c] for r < R; output columns r in [R, Rpad) are zero.
hipError_t launch_transpose_bf16(bf16_t* out, long ldo, const void* in, bool in_f32, long ldi, int R, int C, int Rpad,
                                 hipStream_t s);
hipError_t launch_transpose_f32(float* out, long ldo, const float* in, long ldi, int R, int C, hipStream_t s);
// out[n] (+)= scale * sum_m in[m][n]  (deterministic two-stage; scratch >= colsum_scratch_floats)
long colsum_scratch_floats(int M, int N);
hipError_t launch_colsum(float* out, const void* in, bool in_f32, long ld, int M, int N, float scale, bool accumulate,
                         float* scratch, hipStream_t s);
// LayerNorm backward (eps 1e-5): dres[xrow] (+)= dx; dw, db (+)= column sums (scratch >= ln_bwd_scratch_floats);
// dres_b (nullable): bf16 copy of the updated dres rows; dsum (nullable): = column sums of the updated dres rows
long ln_bwd_scratch_floats(int n, int D);
hipError_t launch_ln_bwd(float* dres, const float* x, const float* dy, long ldy, const float* w, const int* rows, int n,
                         int D, float* dw, float* db, bool accumulate_dx, bool accumulate_dwb, float* scratch,
                         hipStream_t s, bf16_t* dres_b = nullptr, float* dsum = nullptr,
                         const bf16_t* dy_b = nullptr);   // dy_b: bf16 dy (row stride ldy) in place of dy
// out = dh * act'(pre) over [M][N] bf16 and dbias = column sums of out (scratch >= act_bwd_colsum_scratch_floats)
long act_bwd_colsum_scratch_floats(int M, int N);     // (also >= the fused GEMM's (M + 127) / 128 x N)
// out[n] = sum over the nb rows of part[nb][N] (fixed order): the fused GEMM's bias-gradient partials
hipError_t launch_colsum_finish(float* out, const float* part, int nb, int N, hipStream_t s);
hipError_t launch_act_bwd_colsum(bf16_t* out, const bf16_t* pre, const bf16_t* dh, int M, int N, int act, float* dbias,
                                 float* scratch, hipStream_t s);
// dh == nullptr: out = act(pre); else out = dh * act'(pre).  bf16, n % 8 == 0.
hipError_t launch_act(bf16_t* out, const bf16_t* pre, const bf16_t* dh, long n, int act, hipStream_t s);
// attention backward (L <= 80): dqkv [B*L][3*H*64] from qkv (q pre-scaled), O, dO [B*L][H*64]
// dbias (nullable): = column sums of dqkv over all rows (the in_proj bias gradient); bpart: [B][3*H*64] f32 per-caption
// sums; scratch: >= colsum_scratch_floats(max(B, B*L), 3*H*64) floats (both required with dbias)
hipError_t launch_attention_bwd(bf16_t* dqkv, const bf16_t* qkv, const bf16_t* O, const bf16_t* dO, const float* lse,
                                int B, int L, int H, bool causal, hipStream_t s, float* dbias = nullptr,
                                float* bpart = nullptr, float* scratch = nullptr);
int set_attn_bwd_variant(int v);   // 2 = transposed-read kernel (default), 1 = the transposed-copy kernel
// token / positional embedding gradients from dx [B*ctx][D] (dtok fully overwritten)
size_t embed_bwd_scratch_bytes(int B, int ctx, int D);
hipError_t launch_embed_bwd(float* dtok, float* dpos, const float* dx, const int64_t* ids, int B, int ctx, int D,
                            int vocab, void* scratch, size_t scratch_bytes, hipStream_t s);
hipError_t launch_l2norm_bwd(float* du, const float* u, const float* df, int rows, int D, hipStream_t s);
// CE + gradient over rows of z (labels -100 ignored): g = w/count (softmax - onehot); out2[0] += loss,
// out2[1] += sum g z.  rowstat: 2R floats.
hipError_t launch_ce_grad(float* g, const float* z, int R, int C, const int64_t* labels, float wgt_inv_count,
                          float* rowstat, float* out2, hipStream_t s);
hipError_t launch_adamw(float* p, const float* g, float* m, float* v, long n, float lr, float b1, float b2, float eps,
                        float wd, int step, hipStream_t s);
hipError_t launch_weight_from_master(void* out, bool bf16, const float* src, long n, long row_len, long scale_rows,
                                     float scale, hipStream_t s);
hipError_t launch_scale(float* x, long n, float sc, hipStream_t s);
hipError_t launch_cast_bf16(bf16_t* out, const float* in, long n, hipStream_t s);
hipError_t launch_axpy(float* y, const float* x, long n, float a, hipStream_t s);   // y += a x

}  // namespace ce
