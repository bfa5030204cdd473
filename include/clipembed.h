/*
 * clipembed.h — C ABI of the MI355X-native CLIP / PACL / SPARC embedding engine.
 *
 * This is the drop-in boundary for the hot path of lst627/CLIP-Embeds.  Every entry point
 * replaces one reference interface; the citation after each declaration is the reference
 * symbol (path:line, relative to the reference root) whose behaviour it reproduces.
 *
 * Conventions
 *  - Plain C types only; no torch types cross this boundary.
 *  - Every call returns an int status (CE_OK == 0).  On failure ce_last_error() returns a
 *    thread-local, NUL-terminated description of the most recent error on this thread.
 *  - Tensor arguments of the compute calls are DEVICE pointers owned by the caller.  The
 *    library owns its weights and its workspace (allocated per handle, grown on demand,
 *    or up front with ce_reserve()).
 *  - Every compute call is enqueued on `stream` (a hipStream_t, NULL = the null stream) and
 *    returns without a host synchronisation.
 *  - One handle per device.  A handle may be used from any host thread, but calls on one
 *    handle must not overlap in time (they share the handle's workspace); handles on
 *    different devices are fully independent (this is how nn.DataParallel-style callers
 *    drive 8 GPUs from 8 host threads), and so are several handles on one device.
 *  - The library keeps no mutable state outside the handles except the ce_set_* A/B knobs
 *    that take no handle (process-wide atomics, read once per launch; they affect every
 *    handle) and per-device caches keyed by device ordinal (CU count, the kernel-level
 *    entry points' split-K workspace, allocated under a lock).
 */
#ifndef CLIPEMBED_H
#define CLIPEMBED_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum ce_status {
    CE_OK = 0,
    CE_ERR_INVALID = 1,   /* bad argument / shape mismatch / unknown weight name            */
    CE_ERR_HIP = 2,       /* a HIP runtime call failed (message carries hipGetErrorString)    */
    CE_ERR_STATE = 3,     /* weights missing, handle not ready                               */
    CE_ERR_OOM = 4        /* device allocation failed                                        */
};

enum ce_dtype { CE_F32 = 0, CE_BF16 = 1, CE_F16 = 2, CE_I64 = 3, CE_I32 = 4 };

/* Activation of the tower MLPs.  open_clip builds ViT-L-14-336 with exact-erf nn.GELU
 * (open_clip/src/open_clip/model.py:117,193); QuickGELU is the *-quickgelu config flag
 * (transformer.py:32-35). */
enum ce_activation { CE_ACT_GELU_ERF = 0, CE_ACT_QUICK_GELU = 1 };

/* PACL patch weighting (Patch-Aligned-Contrastive-Learning/model/pacl.py:120-145).
 * CE_PACL_ONES reproduces the "Eval only" overwrite at pacl.py:142 (also :193,:272,:288);
 * CE_PACL_SIGMOID10 is sigmoid(10*cos(text, patch)) as used by pacl.py:206-207,:362-363. */
enum ce_pacl_weight { CE_PACL_ONES = 0, CE_PACL_SIGMOID10 = 1 };

/* Where apply_rope (pacl.py:147-181) is applied.  BEFORE = on the 1024-d CLIP patch tokens
 * before the visual projection (open_clip_pacl_rope, pacl.py:184-197); AFTER = on the
 * projected 768-d tokens, used only for the patch activations (open_clip_pacl_rope_after,
 * pacl.py:199-209). */
enum ce_rope { CE_ROPE_NONE = 0, CE_ROPE_BEFORE = 1, CE_ROPE_AFTER = 2 };

typedef struct ce_tower_config {
    int width;       /* D                                  (vision 1024, text 768)         */
    int layers;      /* residual blocks                    (vision 24,   text 12)          */
    int heads;       /* attention heads, head dim = width/heads must be 64                */
    int mlp_width;   /* MLP hidden                         (vision 4096, text 3072)        */
} ce_tower_config;

typedef struct ce_config {
    int embed_dim;          /* output embedding (768)                                      */
    int activation;         /* enum ce_activation                                          */
    int image_size;         /* 336                                                         */
    int patch_size;         /* 14                                                          */
    ce_tower_config vision;
    int context_length;     /* 77                                                          */
    int vocab_size;         /* 49408                                                       */
    ce_tower_config text;
    int pacl_dim;           /* PACL head output dim (768); 0 = no PACL head                */
} ce_config;

/* One host tensor of an open_clip state dict.  `name` is the state-dict key as produced by
 * CLIP.state_dict() (open_clip/src/open_clip/model.py:222-300); the prefixes "module." and
 * "clip_model." (PACL checkpoints, eval_pacl.py:380-388) are stripped.  PACL head keys are
 * "visual_projection.*" / "text_projection.*" as registered by open_clip_pacl
 * (pacl.py:70-79).  data points to host memory, C-contiguous. */
typedef struct ce_tensor {
    const char* name;
    const void* data;
    int dtype;              /* enum ce_dtype: CE_F32, CE_BF16 or CE_F16                    */
    int ndim;
    int64_t shape[4];
} ce_tensor;

typedef struct ce_handle ce_handle;

/* Thread-local description of the last error on the calling thread ("" if none). */
const char* ce_last_error(void);

/* Library version string, e.g. "clipembed 0.1.0 gfx950". */
const char* ce_version(void);

/* Create an engine on HIP device `device`.
 * Replaces: CLIP.__init__ / _build_vision_tower / _build_text_tower
 *   (open_clip/src/open_clip/model.py:105-255) — the tower geometry only; no weights. */
int ce_create(const ce_config* cfg, int device, ce_handle** out);

/* Release the handle and all device memory it owns. */
int ce_destroy(ce_handle* h);

/* Copy (and convert to the engine's device layout) a set of state-dict tensors.
 * May be called several times; later calls overwrite earlier tensors of the same name.
 * Replaces: CLIP.load_state_dict via open_clip.factory.load_checkpoint
 *   (open_clip/src/open_clip/factory.py:171-215); PACL checkpoint loading
 *   (Patch-Aligned-Contrastive-Learning/eval_pacl.py:380-388).
 * Unknown names are an error (CE_ERR_INVALID) unless `allow_unknown` != 0. */
int ce_load_weights(ce_handle* h, const ce_tensor* tensors, int n, int allow_unknown);

/* Number of required CLIP tensors not loaded yet (0 = ready); name of the first one. */
int ce_missing_weights(ce_handle* h, int* n_missing, const char** first_missing);

/* Pre-allocate the workspace for up to `max_images` images and `max_texts` texts per call
 * (optional; compute calls grow it on demand, which synchronises the device once). */
int ce_reserve(ce_handle* h, int max_images, int max_texts);

/* Image tower forward.
 * Replaces: CLIP.encode_image (open_clip/src/open_clip/model.py:279-281) ->
 *   VisionTransformer.forward (transformer.py:825-836): _embeds :701-716, 24 x
 *   ResidualAttentionBlock.forward :257-268, _pool :718-741 ('tok' pool), pooled @ proj.
 * pixels:      device [B,3,image_size,image_size], dtype CE_F32 or CE_BF16, NCHW.
 * out_pooled:  device f32 [B, embed_dim]; L2-normalised when normalize != 0.
 * out_tokens:  optional (NULL = not computed) device [B, grid*grid, width] post-ln_post,
 *              pre-proj patch tokens (transformer.py:738-739,833-834), dtype tokens_dtype
 *              (CE_F32 or CE_BF16). */
int ce_encode_image(ce_handle* h, void* stream, const void* pixels, int pixel_dtype, int B,
                    int normalize, float* out_pooled, void* out_tokens, int tokens_dtype);

/* Text tower forward.
 * Replaces: CLIP.encode_text (open_clip/src/open_clip/model.py:283-301): token_embedding
 *   gather + positional_embedding, 12 causal blocks (mask transformer.py:960-966), ln_final,
 *   argmax (EOT) pooling (transformer.py:839-855), @ text_projection.
 * ids:         device int64 [B, ctx] (ctx must equal context_length).
 * out_pooled:  device f32 [B, embed_dim].
 * out_tokens:  optional device [B, ctx, width] post-ln_final, pre-projection tokens
 *              (model.py:299-300, output_text_tokens=True), dtype tokens_dtype. */
int ce_encode_text(ce_handle* h, void* stream, const int64_t* ids, int B, int ctx,
                   int normalize, float* out_pooled, void* out_tokens, int tokens_dtype);

/* Contrastive logits, fused L2-normalise + scale * I @ T^T.
 * Replaces: CLIP.get_logits (open_clip/src/open_clip/model.py:303-310); the eval scoring
 *   100 * I @ T^T (eval_clip.py:61-63,321-323); ClipLoss.get_logits local-loss slices
 *   (open_clip/src/open_clip/loss.py:155-164; pacl.py:498-501).
 * img [Bi,D], txt [Bt,D] f32 device; out_image_logits [Bi,Bt]; out_text_logits [Bt,Bi]
 * (optional, = transpose).  normalize != 0 L2-normalises rows first (F.normalize, eps 1e-12). */
int ce_get_logits(ce_handle* h, void* stream, const float* img, int Bi, const float* txt,
                  int Bt, int D, float scale, int normalize, float* out_image_logits,
                  float* out_text_logits);

/* Symmetric / NegCLIP contrastive cross-entropy over precomputed logits rows.
 * Replaces: F.cross_entropy(logits, labels) with ignore_index -100 as used by
 *   ClipLoss.forward (open_clip/src/open_clip/loss.py:172-193, labels :113-135) and the
 *   PACL ClipLoss (pacl.py:503-514).
 * logits f32 [R,C] device; labels int64 [R] device (-100 = ignored; any other label outside [0, C),
 * where F.cross_entropy raises, makes the loss NaN: the device values are not read on the host);
 * out_loss: device f32 scalar = mean over non-ignored rows of (logsumexp - logit[label]). */
int ce_cross_entropy(ce_handle* h, void* stream, const float* logits, int R, int C,
                     const int64_t* labels, float* out_loss);

/* PACL visual / text heads (open_clip_pacl.forward_visual / forward_text, pacl.py:112-118;
 * heads :70-79; Patch_Projection :35-48).  Dropout is identity (eval).
 * tokens:   device [B, P, width] CLIP patch tokens (dtype tokens_dtype).
 * rope:     CE_ROPE_NONE or CE_ROPE_BEFORE (apply_rope on the tokens first, pacl.py:187).
 * out_proj: device [B, P, pacl_dim], dtype out_dtype (CE_F32 or CE_BF16). */
int ce_pacl_project_patches(ce_handle* h, void* stream, const void* tokens, int tokens_dtype,
                            int B, int P, int rope, void* out_proj, int out_dtype);
int ce_pacl_project_text(ce_handle* h, void* stream, const float* text_pooled, int B,
                         float* out_proj);

/* Fused PACL patch alignment + pooling + normalisation (pacl.py:120-145, 199-209).
 * visual_proj [Bi,P,Dp] (vp_dtype), text_proj [Bt,Dp] f32.  Broadcast exactly like the
 * reference: R = max(Bi,Bt) output rows, row r uses image (Bi==1?0:r) and text
 * (Bt==1?0:r); Bi and Bt must be equal or one of them 1 (pacl.py:129,143).
 * out_img [R,Dp] = normalize(sum_p w_p v_p), out_txt [Bt,Dp] = normalize(text_proj). */
int ce_pacl_pool(ce_handle* h, void* stream, const void* visual_proj, int vp_dtype, int Bi,
                 int P, const float* text_proj, int Bt, int Dp, int weight_mode, int rope_after,
                 float* out_img, float* out_txt);

/* Whole PACL forward: encode_image(tokens) -> heads -> encode_text -> heads -> pool.
 * Replaces open_clip_pacl.forward / _rope.forward / _rope_after.forward (pacl.py:135-209).
 * rope: enum ce_rope.  out_img [max(Bi,Bt), pacl_dim], out_txt [Bt, pacl_dim] (f32). */
int ce_pacl_forward(ce_handle* h, void* stream, const void* pixels, int pixel_dtype, int Bi,
                    const int64_t* ids, int Bt, int weight_mode, int rope, float* out_img,
                    float* out_txt);

/* SPARC fine-grained alignment (sparc.forward, pacl.py:453-478).
 * v [B,P,D] f32 projected patch embeddings, l [B,T,D] f32 projected token embeddings.
 * out_grouped [B,T,D] = L2norm(rownorm(threshold(minmax(l v^T), sigma)) v);
 * out_l_norm  [B,T,D] = L2norm(l) (optional, may be NULL);
 * out_sim     [B,T,P] optional raw similarity l v^T (may be NULL). */
int ce_sparc_forward(ce_handle* h, void* stream, const float* v, const float* l, int B, int P,
                     int T, int D, float sigma, float* out_grouped, float* out_l_norm,
                     float* out_sim);

/* Eval image preprocessing on the device, replacing the host-side pipelines:
 *   CE_PRE_CLIP_BICUBIC     open_clip/src/open_clip/transform.py:371-389 (image_transform, eval,
 *                           resize_mode 'shortest'): Resize(S, BICUBIC) of the shortest edge with
 *                           Pillow's fixed-point resampler (bit-exact), CenterCrop(S), ToTensor,
 *                           Normalize(OpenAI mean/std, constants.py:1-2)
 *   CE_PRE_PACL_BILINEAR_AA Patch-Aligned-Contrastive-Learning/data/utils.py:33-37: ToTensor,
 *                           Resize((S,S)) bilinear with antialias on the float tensor
 *                           (torch interpolate), Normalize(ImageNet mean/std)
 * images: device uint8 RGB, image b is HWC [heights[b]][widths[b]][3] at images + offsets[b];
 * offsets / heights / widths are HOST arrays of B entries.  S = cfg.image_size.
 * out: device [B,3,S,S] f32 or bf16 (out_dtype), ready for ce_encode_image. */
enum ce_preprocess_mode { CE_PRE_CLIP_BICUBIC = 0, CE_PRE_PACL_BILINEAR_AA = 1 };
int ce_preprocess_images(ce_handle* h, void* stream, const uint8_t* images, const int64_t* offsets,
                         const int* heights, const int* widths, int B, int mode, int out_dtype, void* out);
/* The training transform's resample step (open_clip transform.py:334-355: RandomResizedCrop(S,
 * scale=(0.9, 1.0), BICUBIC) -> ToTensor -> Normalize(OpenAI)); the caller draws the crop boxes on
 * the host (torchvision RandomResizedCrop.get_params with the torch RNG) and the device applies
 * torchvision's F.resized_crop on a PIL image: Pillow's bicubic resampler (bit-exact) from the box
 * (top, left, height, width) of image b to S x S.  boxes: HOST int32 [B][4], inside each image. */
int ce_preprocess_images_boxes(ce_handle* h, void* stream, const uint8_t* images, const int64_t* offsets,
                               const int* heights, const int* widths, const int* boxes, int B, int out_dtype,
                               void* out);

/* SparcLoss.forward (Patch-Aligned-Contrastive-Learning/model/pacl.py:564-584, masked local loss
 * :527-562): global_weight (reference 0.5, :520) * CLIP loss (logit scale 1/temperature) of the
 * L2-normalised means of v_patch over P and of l_tokens over T, + local_weight (reference 1.0,
 * :521) * the mean of the two masked pairwise local losses between
 * grouped and l_tokens.  v_patch f32 [B,P,D] (projected patches, unnormalised), l_tokens f32 [B,T,D]
 * and grouped f32 [B,T,D] (both L2-normalised, as ce_sparc_forward returns them), mask f32 [B,T]
 * (1 = token <= EOT).  out_loss: device f32 [1]. */
int ce_sparc_loss(ce_handle* h, void* stream, const float* v_patch, const float* l_tokens, const float* grouped,
                  const float* mask, int B, int P, int T, int D, float temperature, float global_weight,
                  float local_weight, float* out_loss);

/* The same losses over a global batch sharded across data-parallel ranks.  train_sparc.py:93,105 and
 * train_pacl.py:34-36,95,106 wrap the model in nn.DataParallel: every replica's outputs are gathered to
 * one device and SparcLoss / ClipLoss(0.1) run on the WHOLE batch there.  Here each rank keeps its B
 * samples and the loss value is the reference's global one, in three steps around two collectives the
 * caller issues (RCCL all-gather of the [B,D] features in rank order, RCCL all-reduce (sum) of 5 floats):
 *   ce_sparc_loss_means          out_img / out_txt [B,D] = L2norm(mean_p v_patch), L2norm(mean_t l_tokens)
 *                                (pacl.py:561-562) — the features the ranks all-gather into img_all /
 *                                txt_all [Bg,D];
 *   ce_sparc_loss_partial        parts[5] (device f32, overwritten) = this shard's sums over its rows
 *                                r = row0..row0+B-1 of the global CE both ways (logits 1/temperature *
 *                                img_all[r] . txt_all^T, label r; pacl.py:563-570), then the masked local
 *                                CE sums both ways and the mask count (pacl.py:522-556,575-580) over its
 *                                samples (l_tokens, grouped, mask as for ce_sparc_loss);
 *   ce_contrastive_loss_partial  parts[0..1] as above for the PACL ClipLoss (pacl.py:498-512; features
 *                                already normalised, logit scale `scale`), parts[2..4] = 0;
 *   ce_loss_combine              out_loss = global_weight (P0 + P1) / (2 n_global) + local_weight (P2 + P3)
 *                                / (2 P4) over the all-reduced parts (local_weight 0: no local term).
 * One rank (row0 = 0, B = Bg) gives ce_sparc_loss's value; the shards' sums add up to it in any split. */
int ce_sparc_loss_means(ce_handle* h, void* stream, const float* v_patch, const float* l_tokens, int B, int P, int T,
                        int D, float* out_img, float* out_txt);
int ce_sparc_loss_partial(ce_handle* h, void* stream, const float* img_all, const float* txt_all, int Bg, int row0,
                          const float* l_tokens, const float* grouped, const float* mask, int B, int T, int D,
                          float temperature, float* parts);
int ce_contrastive_loss_partial(ce_handle* h, void* stream, const float* img_all, const float* txt_all, int Bg,
                                int row0, int B, int D, float scale, float* parts);
int ce_loss_combine(ce_handle* h, void* stream, const float* parts, int n_global, float global_weight,
                    float local_weight, float* out_loss);

/* SPARC head training step (Patch-Aligned-Contrastive-Learning/train_sparc.py:29-37,91,106 on
 * model/pacl.py:380-584: sparc / sparc_rope forward in train mode, SparcLoss(temperature), loss.backward(),
 * torch.optim.Adam over the heads; the CLIP towers are frozen, pacl.py:408).  The caller owns f32 master
 * values and gradient slots of the 12 head tensors (visual_projection.0.{weight,bias},
 * .2.linear_projection.0.*, .2.non_linear_projection.{0,2}.*, text_projection.0.*, text_projection.2.*) and
 * runs the optimizer (ce_adamw with weight_decay 0 is torch.optim.Adam).  Data-parallel ranks follow the
 * reference's nn.DataParallel semantics (the loss over the WHOLE gathered batch, gradients summed over
 * replicas) through the same collectives as the value path above.
 *   ce_sparc_train_bind          params / grads: the 12 head tensors by name (f32 device buffers)
 *   ce_sparc_train_sync_weights  engine compute copies of the heads <- masters (after each update)
 *   ce_sparc_train_forward       patch_tokens f32 [B,P,Dv] (visual.output_tokens, ln_post'd), rope:
 *                                CE_ROPE_BEFORE (sparc_rope) or NONE; text f32 [B,T,E] = the text tower's
 *                                tokens (text_mode 0: through text_projection) or the token embeddings
 *                                themselves (text_mode 1: precomputed / LLM embeddings, no text head);
 *                                Dropout(dropout) after both head LayerNorms with masks from a counter
 *                                hash of seed over the element's index in the GLOBAL batch (sample0 =
 *                                this rank's first sample: the masks do not depend on the sharding;
 *                                dropout 0: eval-mode heads).  Keeps every activation the
 *                                backward needs; out_v [B,P,Pd], out_l [B,T,Pd] (normalised), out_g
 *                                [B,T,Pd] (normalised grouped patches) as sparc.forward returns them
 *                                (each nullable).  T <= 80.
 *   ce_sparc_train_loss_grad     after ce_sparc_loss_means(out_v, out_l) and the all-gather of those
 *                                means (img_all / txt_all [Bg,Pd], this rank's rows at row0): parts[5]
 *                                (as ce_sparc_loss_partial, for ce_loss_combine after the all-reduce) and
 *                                the gradient of the global loss w.r.t. this rank's means and local-term
 *                                inputs (kept in the handle); mask f32 [B,T]; mask_total = the mask's sum
 *                                over the global batch (the local term's divisor).
 *   ce_sparc_train_backward      every bound gradient slot (overwritten; the text head's are zeroed with
 *                                text_mode 1) from those gradients through the alignment, the heads, the
 *                                dropouts and the head LayerNorms. */
int ce_sparc_train_bind(ce_handle* h, const ce_tensor* params, const ce_tensor* grads, int n);
int ce_sparc_train_sync_weights(ce_handle* h, void* stream);
int ce_sparc_train_forward(ce_handle* h, void* stream, const float* patch_tokens, int B, int P, int rope,
                           const float* text, int text_mode, int T, float sigma, float dropout, uint64_t seed,
                           int64_t sample0, float* out_v, float* out_l, float* out_g);
int ce_sparc_train_loss_grad(ce_handle* h, void* stream, const float* img_all, const float* txt_all, int Bg, int row0,
                             const float* mask, float mask_total, float temperature, float global_weight,
                             float local_weight, float* parts);
int ce_sparc_train_backward(ce_handle* h, void* stream);

/* apply_rope (pacl.py:147-181): de-interleaving rotary embedding over positions 0..P-1.
 * x, out: device f32 [B,P,D] (may alias). */
int ce_apply_rope(ce_handle* h, void* stream, const float* x, int B, int P, int D, float* out);

/* Kernel timing for roofline reporting: when enabled, every launch of the GEMM / attention
 * / LayerNorm kernels is bracketed by HIP events on its stream and the elapsed times are
 * accumulated per kernel tag.  ce_kernel_stats reads them (after a stream sync). */
int ce_set_kernel_timing(ce_handle* h, int enable);
/* Restrict timing to the launches whose tag equals `tag` (NULL or "" = all tags): the bench brackets
 * only the dominant kernel inside its timed region, so the events do not perturb the step time. */
int ce_set_kernel_timing_filter(ce_handle* h, const char* tag);
int ce_kernel_stats(ce_handle* h, int index, char* name, int name_len, double* total_ms,
                    int64_t* launches, double* flops, double* bytes);

/* ---- kernel-level entry points (parity tests, micro-benchmarks); no handle, device = current ----
 * GEMM: out = act(A W^T + bias) + resid.  A [M,K] bf16, W [N,K] bf16 (nn.Linear layout), bias f32 [N]
 * (nullable), resid f32 [M,N] (nullable), out [M,N] f32 or bf16.  K % 64 == 0, N % 64 == 0.
 * act: 0 none, 1 GELU(erf), 2 QuickGELU.  (ResidualAttentionBlock linears, transformer.py:228-239) */
int ce_kernel_gemm_bf16(void* stream, const void* A, const void* W, int M, int N, int K, const float* bias,
                        int act, const float* resid, void* out, int out_dtype);
/* Select the GEMM main-loop schedule for subsequent launches (bits 0-7: 1 = the default shape policy
 * (ce_set_gemm_auto: the 4-phase kernel, SCHED 1, or the four-wave persistent kernels by shape), 11 =
 * the four-wave persistent kernel (SCHED 11) wherever its epilogues apply (bf16 without residual,
 * f32 LN statistics, plain f32), other values select 1; bits 8-15: tile-order M-group, 0 = keep;
 * bits 24-30: 1 + first-round stagger in units of s_sleep 127 (~8k cycles) for half the CUs, 0 =
 * keep).  The fields change together (one atomic word).  Returns the previous schedule | M-group << 8.
 * For A/B measurement.  (The other schedules of rounds 1-5 were measured slower and removed in
 * round 6) */
int ce_set_gemm_schedule(int schedule);
/* Split-K tail of the GEMM (default on): when a grid's last round holds few tiles, those tiles are
 * computed as K-chunks summed by a fixup launch.  Returns the previous setting.  For A/B. */
int ce_set_gemm_splitk(int enable);
/* Shape policy of the default GEMM schedule (env CE_GEMM_AUTO at first use): 0 = every GEMM on
 * the 4-phase schedule (with its split-K tail), 1 = the default (grids of >= 4 tiles per CU with
 * no residual, i.e. the vision QKV and c_fc GEMMs, on the four-wave persistent schedule),
 * 2 = every large grid on it, 3 = large grids without a residual.  Returns the previous mode.
 * Runtime A/B of the bench configuration against the plain path in one process (parity tests). */
int ce_set_gemm_auto(int mode);
/* GEMM kernel-variant bits for A/B measurement (env CE_GEMM_VARIANT at first use; a negative value
 * restores the default, bits 0|1|7|8|9|13): bit 0 = the four-wave persistent schedule does not drain
 * an epilogue's stores at the next tile's first K-tile; bit 1 = its epilogues written for one wave per
 * SIMD (operands staged in LDS, clipped buffer stores; also lets the default policy put GELU GEMMs on
 * that schedule; off: those GEMMs run on SCHED 1); bit 4 = one tile per four-wave workgroup; bit 5 =
 * split-K tail on the four-wave schedule; bit 7 = the hi/lo residual GEMMs (epi 3, N % 256 == 0, grids
 * of >= 2 tiles per CU, default policy) on the staged-residual four-wave kernel;
 * bits 8 / 9 (a K-tile's operand DMAs spread over B2 and B3) are always on since
 * round 6; bit 13 = the caller's small one-tile grids (text tower) on the four-wave kernels.
 * Returns the previous bits. */
int ce_set_gemm_variant(int bits);
/* Attention-forward variant for A/B: 381 (default) = fixed-offset key tiles
 * (once tile 0's row maxima lie within +-64 log2 units: no row max, no offset, overflow-checked row
 * sums, an overflowing tile redone on the general online-softmax path), one barrier per key tile,
 * 16-B output stores, V^T fragments by inline-asm ds_read_b64_tr_b16, K/V DMAs through row-clipped
 * buffer descriptors, and key 0 folded into O / l before the key tiles, which then cover keys 1..L-1
 * (non-causal L with (L - 1) % 64 == 0: L = 577 runs 9 full tiles, no single-key masked tile); 125 =
 * the same without key 0 first (also what 381 runs for other L).  Anything else selects 381.  Causal
 * launches (text tower) run the general-path kernel with the same loads and stores (88).  (The other
 * variants of rounds 1-5 were measured slower and removed in round 6)
 * Returns the previous variant. */
int ce_set_attn_variant(int var);
/* Attention-backward kernel of the text-tower training for A/B (env CE_ATTN_BWD at first use): 3 = the
 * default: the transposed-read kernel with the causal structure used (only the score tiles on or below
 * the diagonal, contractions over the blocks that can be non-zero) and the outputs written as whole
 * rows from LDS; 2 = the transposed-read kernel over every tile (operands contracted over their image's
 * row index come from ds_read_b64_tr_b16, 73 KB of LDS, two workgroups per CU); 1 = the kernel with
 * transposed LDS copies (136 KB, one per CU).  Returns the previous setting. */
int ce_set_attn_bwd_variant(int v);
/* Weight-gradient GEMM with MN-major operands: C[m][n] = scale_m * sum_k A[k][m] B[k][n]
 * with A [K][lda], B [K][ldb] bf16 row-major (the activations of a linear layer's input and output
 * gradient, reduction over their rows), C [M][ldc] f32, scale_m = scale for m < scale_rows else 1.
 * M % 256 == 0, N % 256 == 0, lda >= M, ldb >= N (multiples of 8), 16-B aligned.  The text-tower
 * backward's dW of in_proj / out_proj / c_fc / c_proj (autograd of transformer.py:228-239). */
int ce_kernel_gemm_tn_bf16(void* stream, const void* A, int64_t lda, const void* B, int64_t ldb, int M, int N, int K,
                           float* C, int64_t ldc, int scale_rows, float scale);
/* Text-tower training: weight gradients by the MN-major GEMM above (1, default) or by transposed
 * operand copies and the forward GEMM (0, the round-3 path).  Returns the previous setting.  For A/B. */
int ce_set_train_dw_tn(int on);
/* Text-tower training: the MLP's activation backward (dpre = dh * act'(pre)) and the c_fc bias
 * gradient in the epilogue of the dX GEMM that produces dh (1, default, where the four-wave kernel
 * takes that GEMM) or as a separate kernel over the GEMM's bf16 output (0).  Same dpre values; the
 * bias sums differ in f32 summation order only.  Returns the previous setting.  For A/B. */
int ce_set_train_act_bwd_fuse(int on);
/* f32 GEMM kernel of the projections, logits and SPARC einsums (pacl.py:460,472): 1 = the
 * register-blocked 96 x 128 kernel (default; 16-B aligned operands with K % 4 == 0); 2 = as 1, and
 * for batched products of M <= 80 rows and N >= 192 (SPARC's T = 77 rows per sample) the 80 x 192
 * short-M kernel on v_mfma_f32_16x16x4_f32; 0 = the 64 x 64 scalar-staged kernel.  Returns the
 * previous setting.  For A/B and parity tests. */
int ce_set_fgemm_variant(int v);
/* Launch counters per GEMM kernel path since the last reset: counts[path + epi] with path 0 =
 * four-wave persistent (SCHED 11), 3 = 4-phase (SCHED 1), 6 = split-K tail fixup, 9 / 10 = unused
 * since round 6 (removed schedules), and epi 0 = plain, 1 = LN statistics, 2 = LN fold.  n <= 13
 * entries are written. */
int ce_gemm_path_counts(int64_t* counts, int n, int reset);
/* GEMM with an LN-fold / LN-stats epilogue (the folded ResidualAttentionBlock,
 * transformer.py:257-268), as the engine launches it:
 *   epi 1 (LN stats): out f32 = A W^T + bias + resid; xb = bf16(out); stats_part[m][n/64] = (mean,
 *         sum of squared deviations) of row m's 64-column slab n/64.  act must be 0.
 *   epi 2 (LN fold):  out bf16 = act(fold_stats[m].y * (A W^T - fold_stats[m].x * fold_c[n]) + bias[n]).
 *   epi 3 (LN stats, hi/lo residual stream): resid = bf16 planes [2][M][N] (value = hi + lo); the
 *         output v = A W^T + bias + resid goes to xb as planes [2][M][N], hi = bf16(v), lo =
 *         bf16(v - hi) (out unused); stats_part as epi 1.
 *   epi 4 (hi/lo residual, f32 out): out f32 = A W^T + bias + (hi + lo) of the resid planes.
 * epi 0 is ce_kernel_gemm_bf16. */
int ce_kernel_gemm_bf16_epi(void* stream, const void* A, const void* W, int M, int N, int K, const float* bias,
                            int act, const float* resid, void* out, int out_dtype, int epi, void* xb,
                            void* stats_part, const void* fold_stats, const float* fold_c);
/* Diagnostics: when buf (device, n_blocks x 4 uint64) is non-null, the GEMM kernels record per workgroup {s_memrealtime at start, after the K-loop, after wave 0's epilogue,
 * (XCC id << 32) | HW_ID} for blocks < n_blocks.  Null turns it off.  The pointer is process-wide
 * and every later GEMM launch of every handle and stream writes through it: diagnostics only, one
 * stream at a time, and call ce_set_gemm_trace(NULL, 0) (after a sync) before freeing buf. */
int ce_set_gemm_trace(void* buf, int64_t n_blocks);
/* (mu, rstd) per row (eps 1e-5) from nslab 64-column slab statistics of an LN-stats GEMM:
 * stats [rows] float2, part [rows][nslab] float2. */
int ce_kernel_ln_stats_finalize(void* stream, void* stats, const void* part, int rows, int nslab);
/* LayerNorm folding of both towers (default on; env CE_LN_FOLD=0 turns it off at ce_create):
 * ln_1/ln_2 of every block are folded into the in_proj/c_fc weights at ce_load_weights, and the
 * residual GEMMs emit the row statistics, so no LayerNorm launch remains inside the blocks
 * (the text tower's entry state comes from the token-embedding kernel).  Needs each
 * block's in_proj/c_fc weight+bias and ln_1/ln_2 loaded in one ce_load_weights call; otherwise
 * that tower runs unfolded (also the text tower after ce_train_sync_weights, until it is loaded
 * again).  *previous (may be null) gets the previous setting. */
int ce_set_ln_fold(ce_handle* h, int enable, int* previous);
/* Residual stream of the LN-folded towers as two bf16 planes (default on; env CE_RESID_HL=0 at
 * ce_create): inside the blocks the out-proj / c_proj GEMMs read x = hi + lo and write hi = bf16(x),
 * lo = bf16(x - hi) (hi doubles as the folded GEMMs' bf16 operand) instead of f32 x plus its bf16
 * copy: 4 B per element written instead of 6; |x - (hi + lo)| <= 2^-16 |x|.  The tower's last
 * residual GEMM writes f32 x.  *previous (may be null) gets the previous setting. */
int ce_set_resid_hl(ce_handle* h, int enable, int* previous);
/* Pooled-only encode calls (out_tokens null; the PACL text tower) run each tower's last block for
 * the pooled rows only — the CLS row of every image, the EOT (argmax id) row of every caption —
 * since no other row of that block reaches the output (transformer.py:718-741, model.py:295-299).
 * Default on with the LN-folded hi/lo towers (env CE_POOLED_PRUNE=0 at ce_create turns it off);
 * *previous (may be null) gets the previous setting. */
int ce_set_pooled_prune(ce_handle* h, int enable, int* previous);
/* Attention core over packed qkv [B*L, 3*H*64] bf16 -> out [B*L, H*64] bf16 (transformer.py:242-255). */
int ce_kernel_attention(void* stream, const void* qkv, void* out, int B, int L, int H, int causal);
/* LayerNorm rows [rows, D] f32 -> f32/bf16 (eps 1e-5; transformer.py:23-29).  D % 256 == 0. */
int ce_kernel_layernorm(void* stream, const float* in, void* out, int out_dtype, const float* w,
                        const float* b, int rows, int D);

/* ---- Text-tower training: the open_clip NegCLIP step with a locked image tower
 * (open_clip_train/train.py:85-189, main.py:271-302; train-clip.sh: --lock-image --local-loss
 * --gather-with-grad [--usehardtext]).  The caller owns f32 master values and gradient slots
 * (device buffers, e.g. views of flat torch tensors so RCCL can all-reduce them in one call):
 *
 *   ce_train_bind          every text tensor (token_embedding.weight, positional_embedding,
 *                          transformer.resblocks.*, ln_final.*, text_projection) -> {param, grad}
 *   ce_train_sync_weights  engine compute copies (bf16 matrices, f32 vectors) <- masters
 *   ce_text_forward_train  CLIP.encode_text(normalize=True) keeping the activations the
 *                          backward needs; out_features [B][embed] f32 (nullable)
 *   ce_text_backward       d loss / d features [B][embed] -> every bound gradient slot
 *                          (overwritten), through F.normalize, projection, ln_final on the EOT
 *                          rows, the blocks (attention: causal, context <= 80) and the embeddings
 *   ce_contrastive_grad    z = scale A B^T; CE over rows (labels -100 ignored, loss.py:127-135);
 *                          out2[0] += weight * inv_count * sum CE, out2[1] += sum G o z
 *                          (= d loss / d logit_scale); dA += scale G B, dB += scale G^T A
 *                          (nullable), G = weight * inv_count * (softmax - onehot)
 *   ce_adamw               torch.optim.AdamW over one flat f32 group (step counts from 1) */
int ce_train_bind(ce_handle* h, const ce_tensor* params, const ce_tensor* grads, int n);
int ce_train_sync_weights(ce_handle* h, void* stream);
int ce_text_forward_train(ce_handle* h, void* stream, const int64_t* ids, int B, float* out_features);
int ce_text_backward(ce_handle* h, void* stream, const float* d_features, int B);
/* ce_text_backward that also records hipEvent_t events[i] (n_events <= text layers + 1, null entries
 * skipped) on the stream as the gradients become final: events[0] after the head (ln_final,
 * text_projection), events[1 + i] after block (layers - 1 - i), the blocks running top-down; the
 * token / positional embeddings are final at the end.  Lets the caller all-reduce finished buckets of
 * blocks on another stream while the lower blocks' backward runs (DDP's bucketed overlap,
 * open_clip_train/main.py:302). */
int ce_text_backward_events(ce_handle* h, void* stream, const float* d_features, int B, void* const* events,
                            int n_events);
int ce_contrastive_grad(ce_handle* h, void* stream, const float* A, int Ra, const float* B, int Cb, int E, float scale,
                        const int64_t* labels, float weight, float inv_count, float* out2, float* dA, float* dB);
int ce_adamw(void* stream, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float lr,
             float beta1, float beta2, float eps, float weight_decay, int step);

/* ---- CLIP BPE tokenizer (host; replaces open_clip SimpleTokenizer, tokenizer.py:133-265) ----
 * `merges` is the DECOMPRESSED text of bpe_simple_vocab_16e6.txt.gz (tokenizer.py:144: header
 * line, then "a b" merge lines); extra specials follow <start_of_text>, <end_of_text>
 * (tokenizer.py:151-154).  Text passed in is already cleaned (ftfy / html.unescape / whitespace /
 * lower: tokenizer.py:66-90 -- done by the Python host layer); UTF-8.  Status 0 = ok, else see
 * ce_tokenizer_last_error(). */
typedef struct ce_tokenizer ce_tokenizer;
int ce_tokenizer_create(const char* merges, size_t len, const char* const* extra_special, int n_extra,
                        ce_tokenizer** out);
int ce_tokenizer_destroy(ce_tokenizer* t);
const char* ce_tokenizer_last_error(void);
int ce_tokenizer_vocab_size(const ce_tokenizer* t);
int ce_tokenizer_special_ids(const ce_tokenizer* t, int32_t* sot, int32_t* eot);
/* SimpleTokenizer.encode (tokenizer.py:213-219): ids of one text, no SOT/EOT.  Writes
 * min(n, cap) ids; *n_out = n (call with ids = NULL to size the buffer). */
int ce_tokenizer_encode(ce_tokenizer* t, const char* text, int32_t* ids, int cap, int* n_out);
/* SimpleTokenizer.__call__ (tokenizer.py:226-265): out[n][context_length] int64 = SOT + ids + EOT,
 * truncated with the last id forced to EOT, zero padded. */
int ce_tokenize(ce_tokenizer* t, const char* const* texts, int n, int context_length, int64_t* out);
/* SimpleTokenizer.decode (tokenizer.py:221-224); *len_out = byte length, buf NUL-terminated. */
int ce_tokenizer_decode(const ce_tokenizer* t, const int32_t* ids, int n, char* buf, int cap, int* len_out);

#ifdef __cplusplus
}
#endif
#endif /* CLIPEMBED_H */
