// C ABI of libclipembed (include/clipembed.h): weight registry, workspace, tower orchestration.
//
// The tower forward mirrors open_clip (reference paths relative to the reference root):
//   VisionTransformer.forward   open_clip/src/open_clip/transformer.py:825-836
//     _embeds :701-716  (conv1 -> +cls -> +pos -> ln_pre)
//     24 x ResidualAttentionBlock.forward :257-268  (x += attn(ln_1 x); x += mlp(ln_2 x))
//     _pool :718-741 ('tok': ln_post on all tokens, pooled = row 0), pooled @ proj
//   CLIP.encode_text            open_clip/src/open_clip/model.py:283-301
//   CLIP.get_logits             model.py:303-310
// The residual stream is kept in f32 in HBM; every GEMM reads bf16 activations and bf16
// weights and accumulates in f32 (MFMA); LayerNorm statistics are f32.
#include "../../include/clipembed.h"
#include "ce_kernels.h"
#include "knobs.h"

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

using ce::bf16_t;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                             \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return fail(CE_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),         \
                        __FILE__, __LINE__);                                                      \
    } while (0)

#define CE_TRY(expr)                     \
    do {                                 \
        int rc_ = (expr);                \
        if (rc_ != CE_OK) return rc_;    \
    } while (0)

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

enum Store { ST_F32, ST_BF16, ST_BF16_PADK, ST_F32_T, ST_SCALAR };

struct WSpec {
    std::vector<int64_t> shape;
    Store st;
    bool required;   // required for the CLIP towers
};

inline uint16_t host_f2bf(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
inline float host_bf2f(uint16_t v) {
    uint32_t u = (uint32_t)v << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}
inline float host_h2f(uint16_t h) {
    const uint32_t sign = (uint32_t)(h & 0x8000) << 16;
    uint32_t exp = (h >> 10) & 0x1f, man = h & 0x3ff, u;
    if (exp == 0) {
        if (man == 0) u = sign;
        else {
            exp = 127 - 15 + 1;
            while (!(man & 0x400)) { man <<= 1; --exp; }
            man &= 0x3ff;
            u = sign | (exp << 23) | (man << 13);
        }
    } else if (exp == 31) {
        u = sign | 0x7f800000u | (man << 13);
    } else {
        u = sign | ((exp + 127 - 15) << 23) | (man << 13);
    }
    float f;
    memcpy(&f, &u, 4);
    return f;
}

struct Blk {
    const float *ln1w, *ln1b, *bqkv, *bout, *ln2w, *ln2b, *bfc, *bproj;
    const bf16_t *wqkv, *wout, *wfc, *wproj;
};

struct KStat {
    std::string name;
    double ms = 0, flops = 0, bytes = 0;
    int64_t n = 0;
};
struct Pending {
    int tag;
    hipEvent_t a, b;
};

}  // namespace

struct ce_handle {
    ce_config cfg{};
    int device = 0;
    std::map<std::string, WSpec> specs;
    std::map<std::string, std::string> alias;
    std::map<std::string, void*> dptr;
    std::map<std::string, bool> loaded;
    float logit_scale = std::log(1.0f / 0.07f);
    int Kp = 0;      // padded patch K
    int G = 0;       // patch grid side
    // workspace
    char* ws = nullptr;      // vision tower (and PACL / sequential paths)
    size_t ws_bytes = 0;
    char* ws_t = nullptr;    // text tower: its own buffers, so encode_text may run on another stream
    size_t ws_t_bytes = 0;   // concurrently with encode_image
    char* tmp = nullptr;
    size_t tmp_bytes = 0;
    char* pool = nullptr;        // PACL pooling: per-split partial rows
    size_t pool_bytes = 0;
    float* scratch = nullptr;    // 256 B
    // device preprocessing: tap tables (pinned host staging -> device), intermediate rows
    char* prep_host = nullptr;
    size_t prep_host_bytes = 0;
    char* prep_dev = nullptr;
    size_t prep_dev_bytes = 0;
    char* prep_tmp = nullptr;
    size_t prep_tmp_bytes = 0;
    hipEvent_t prep_ev = nullptr;    // the staging buffer's last upload
    // RoPE tables (pacl.py:147-181): [P][D/2] for D = vision width and D = pacl_dim
    float *rc_v = nullptr, *rs_v = nullptr, *rc_p = nullptr, *rs_p = nullptr;
    // timing
    bool timing = false;
    std::string timing_only;     // non-empty: only launches with this tag are bracketed
    float* cur_part = nullptr;   // GEMM split-K slabs of the tower whose launches are being issued
    // packed text rows (pooled-only calls): the sequence offsets of the last launch, read back on the
    // host during a full profile pass only (every launch timed, no filter), so that the per-kernel
    // table carries the packed launches' work; seg_dev identifies the device copy they describe
    std::vector<int> seg_host;
    const int* seg_dev = nullptr;
    // LayerNorm folding of the vision blocks: enabled unless CE_LN_FOLD=0 /
    // ce_set_ln_fold(h, 0); folded[name] = "<name>@fold{,_c,_d}" are current for weight `name`
    bool ln_fold = true;
    // folded image tower: residual stream inside the blocks as hi/lo bf16 planes (EPI_LN_STATS_HL;
    // env CE_RESID_HL=0 keeps the f32 stream + bf16 copy)
    bool resid_hl = true;
    // pooled-only calls (no tokens requested): the last block of each tower runs for the pooled
    // rows only (CLS / EOT); env CE_POOLED_PRUNE=0 / ce_set_pooled_prune(h, 0)
    bool pooled_prune = true;
    std::map<std::string, bool> folded;
    // text-tower training: caller-owned f32 master values and gradient slots per
    // trainable tensor (device pointers), saved activations of the last ce_text_forward_train
    std::map<std::string, std::pair<float*, float*>> bound;
    char* tr = nullptr;
    size_t tr_bytes = 0;
    int tr_B = 0;                // batch of the saved activations (0 = none)
    // SPARC head training (ce_sparc_train_*): caller-owned f32 masters / gradient slots of the 12 head
    // tensors, the saved activations of the last ce_sparc_train_forward and its settings
    std::map<std::string, std::pair<float*, float*>> sp_bound;
    char* sp = nullptr;
    size_t sp_bytes = 0;
    int sp_B = 0, sp_P = 0, sp_T = 0, sp_text = 0, sp_state = 0;   // state: 1 forward done, 2 loss grad done
    float sp_sigma = 0.f, sp_drop = 0.f;
    uint64_t sp_seed = 0;
    int64_t sp_sample0 = 0;
    std::vector<KStat> stats;
    std::map<std::string, int> stat_idx;
    std::vector<Pending> pending;
    std::vector<hipEvent_t> free_ev;
};

namespace {

// ---------------------------------------------------------------------------------------------
// weight registry
void add_block_specs(ce_handle* h, const std::string& p, int D, int F) {
    auto& s = h->specs;
    s[p + "ln_1.weight"] = {{D}, ST_F32, true};
    s[p + "ln_1.bias"] = {{D}, ST_F32, true};
    s[p + "attn.in_proj_weight"] = {{3 * D, D}, ST_BF16, true};
    s[p + "attn.in_proj_bias"] = {{3 * D}, ST_F32, true};
    s[p + "attn.out_proj.weight"] = {{D, D}, ST_BF16, true};
    s[p + "attn.out_proj.bias"] = {{D}, ST_F32, true};
    s[p + "ln_2.weight"] = {{D}, ST_F32, true};
    s[p + "ln_2.bias"] = {{D}, ST_F32, true};
    s[p + "mlp.c_fc.weight"] = {{F, D}, ST_BF16, true};
    s[p + "mlp.c_fc.bias"] = {{F}, ST_F32, true};
    s[p + "mlp.c_proj.weight"] = {{D, F}, ST_BF16, true};
    s[p + "mlp.c_proj.bias"] = {{D}, ST_F32, true};
}

void build_specs(ce_handle* h) {
    const ce_config& c = h->cfg;
    auto& s = h->specs;
    const int Dv = c.vision.width, Dt = c.text.width, E = c.embed_dim;
    const int Lv = h->G * h->G + 1;
    s["visual.class_embedding"] = {{Dv}, ST_F32, true};
    s["visual.positional_embedding"] = {{Lv, Dv}, ST_F32, true};
    s["visual.proj"] = {{Dv, E}, ST_F32, true};
    s["visual.conv1.weight"] = {{Dv, 3, c.patch_size, c.patch_size}, ST_BF16_PADK, true};
    s["visual.ln_pre.weight"] = {{Dv}, ST_F32, true};
    s["visual.ln_pre.bias"] = {{Dv}, ST_F32, true};
    s["visual.ln_post.weight"] = {{Dv}, ST_F32, true};
    s["visual.ln_post.bias"] = {{Dv}, ST_F32, true};
    for (int i = 0; i < c.vision.layers; ++i)
        add_block_specs(h, "visual.transformer.resblocks." + std::to_string(i) + ".", Dv, c.vision.mlp_width);
    s["token_embedding.weight"] = {{c.vocab_size, Dt}, ST_F32, true};
    s["positional_embedding"] = {{c.context_length, Dt}, ST_F32, true};
    s["text_projection"] = {{Dt, E}, ST_F32, true};
    s["ln_final.weight"] = {{Dt}, ST_F32, true};
    s["ln_final.bias"] = {{Dt}, ST_F32, true};
    for (int i = 0; i < c.text.layers; ++i)
        add_block_specs(h, "transformer.resblocks." + std::to_string(i) + ".", Dt, c.text.mlp_width);
    s["logit_scale"] = {{}, ST_SCALAR, false};
    if (c.pacl_dim > 0) {
        const int Pd = c.pacl_dim;
        // open_clip_pacl heads, pacl.py:70-79 (Sequential(LayerNorm, Dropout, Patch_Projection))
        s["visual_projection.0.weight"] = {{Dv}, ST_F32, false};
        s["visual_projection.0.bias"] = {{Dv}, ST_F32, false};
        s["visual_projection.2.linear_projection.0.weight"] = {{Pd, Dv}, ST_BF16, false};
        s["visual_projection.2.linear_projection.0.bias"] = {{Pd}, ST_F32, false};
        s["visual_projection.2.non_linear_projection.0.weight"] = {{Pd, Dv}, ST_BF16, false};
        s["visual_projection.2.non_linear_projection.0.bias"] = {{Pd}, ST_F32, false};
        s["visual_projection.2.non_linear_projection.2.weight"] = {{Pd, Pd}, ST_BF16, false};
        s["visual_projection.2.non_linear_projection.2.bias"] = {{Pd}, ST_F32, false};
        s["text_projection.0.weight"] = {{E}, ST_F32, false};
        s["text_projection.0.bias"] = {{E}, ST_F32, false};
        s["text_projection.2.weight"] = {{Pd, E}, ST_F32_T, false};
        s["text_projection.2.bias"] = {{Pd}, ST_F32, false};
        // Patch_Projection registers the same Sequential twice (pacl.py:39)
        h->alias["visual_projection.2.text_projection.0.weight"] = "visual_projection.2.linear_projection.0.weight";
        h->alias["visual_projection.2.text_projection.0.bias"] = "visual_projection.2.linear_projection.0.bias";
    }
}

std::string canonical(const ce_handle* h, const char* raw) {
    std::string n(raw);
    for (;;) {
        if (n.rfind("module.", 0) == 0) n = n.substr(7);
        else if (n.rfind("clip_model.", 0) == 0) n = n.substr(11);
        else break;
    }
    auto it = h->alias.find(n);
    if (it != h->alias.end()) return it->second;
    return n;
}

template <class T = float>
const T* W(const ce_handle* h, const std::string& n) {
    auto it = h->dptr.find(n);
    return it == h->dptr.end() ? nullptr : static_cast<const T*>(it->second);
}

Blk block_ptrs(const ce_handle* h, const std::string& p) {
    Blk b;
    b.ln1w = W(h, p + "ln_1.weight");
    b.ln1b = W(h, p + "ln_1.bias");
    b.bqkv = W(h, p + "attn.in_proj_bias");
    b.bout = W(h, p + "attn.out_proj.bias");
    b.ln2w = W(h, p + "ln_2.weight");
    b.ln2b = W(h, p + "ln_2.bias");
    b.bfc = W(h, p + "mlp.c_fc.bias");
    b.bproj = W(h, p + "mlp.c_proj.bias");
    b.wqkv = W<bf16_t>(h, p + "attn.in_proj_weight");
    b.wout = W<bf16_t>(h, p + "attn.out_proj.weight");
    b.wfc = W<bf16_t>(h, p + "mlp.c_fc.weight");
    b.wproj = W<bf16_t>(h, p + "mlp.c_proj.weight");
    return b;
}

int check_ready(ce_handle* h, bool need_pacl) {
    for (auto& kv : h->specs) {
        const bool pacl = kv.first.rfind("visual_projection.", 0) == 0 || kv.first.rfind("text_projection.", 0) == 0;
        if ((kv.second.required || (need_pacl && pacl)) && !h->loaded[kv.first])
            return fail(CE_ERR_STATE, "weight '%s' has not been loaded", kv.first.c_str());
    }
    return CE_OK;
}

// ---------------------------------------------------------------------------------------------
// timing
int stat_tag(ce_handle* h, const char* name) {
    auto it = h->stat_idx.find(name);
    if (it != h->stat_idx.end()) return it->second;
    const int idx = (int)h->stats.size();
    h->stats.push_back(KStat{name});
    h->stat_idx[name] = idx;
    return idx;
}

hipEvent_t get_event(ce_handle* h) {
    if (!h->free_ev.empty()) {
        hipEvent_t e = h->free_ev.back();
        h->free_ev.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

template <class F>
int timed(ce_handle* h, hipStream_t s, const char* name, double flops, double bytes, F&& launch) {
    if (!h->timing || (!h->timing_only.empty() && h->timing_only != name)) {
        hipError_t e = launch();
        if (e != hipSuccess) return fail(CE_ERR_HIP, "%s launch failed: %s", name, hipGetErrorString(e));
        return CE_OK;
    }
    const int tag = stat_tag(h, name);
    hipEvent_t a = get_event(h), b = get_event(h);
    (void)hipEventRecord(a, s);
    hipError_t e = launch();
    (void)hipEventRecord(b, s);
    if (e != hipSuccess) return fail(CE_ERR_HIP, "%s launch failed: %s", name, hipGetErrorString(e));
    h->pending.push_back({tag, a, b});
    h->stats[tag].flops += flops;
    h->stats[tag].bytes += bytes;
    h->stats[tag].n += 1;
    return CE_OK;
}

int resolve_pending(ce_handle* h) {
    for (auto& p : h->pending) {
        HIP_TRY(hipEventSynchronize(p.b));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, p.a, p.b));
        h->stats[p.tag].ms += ms;
        h->free_ev.push_back(p.a);
        h->free_ev.push_back(p.b);
    }
    h->pending.clear();
    return CE_OK;
}

// ---------------------------------------------------------------------------------------------
// workspace
size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct TowerWs {
    float* x;
    bf16_t *xn, *qkv, *att, *hid;
    bf16_t* xlo;          // lo plane right after xn (hi/lo residual stream: plane stride rows * D)
    float* pooled;
    int* rows;
    int* seg;             // packed text rows (pooled-only calls): [B + 1] offsets, seg[B] = live rows
    float* part;     // GEMM split-K partial tiles (ce::kGemmPartElems f32), per tower: the towers may
                     // run concurrently on two streams
    float2* stats;        // LN folding: (mu, rstd) per row of the residual stream
    float2* stats_part;   // LN folding: per-64-column-slab (mean, M2) from the residual GEMMs
};

size_t tower_bytes(long rows, int D, int F, long extra_hid_elems, long B) {
    size_t n = 0;
    n += align256(rows * D * 4);
    n += align256(2 * rows * D * 2);
    n += align256(rows * 3 * D * 2);
    n += align256(rows * D * 2);
    n += align256(std::max(rows * F, extra_hid_elems) * 2);
    n += align256(B * D * 4);
    n += align256((2 * B + 1) * 4);
    n += align256(ce::kGemmPartElems * 4);
    n += align256(rows * 8);
    n += align256(rows * (D / 64) * 8);
    return n;
}

TowerWs carve(char* base, long rows, int D, int F, long extra_hid_elems, long B) {
    TowerWs w;
    char* p = base;
    w.x = (float*)p; p += align256(rows * D * 4);
    w.xn = (bf16_t*)p;
    w.xlo = w.xn + rows * D;
    p += align256(2 * rows * D * 2);
    w.qkv = (bf16_t*)p; p += align256(rows * 3 * D * 2);
    w.att = (bf16_t*)p; p += align256(rows * D * 2);
    w.hid = (bf16_t*)p; p += align256(std::max(rows * F, extra_hid_elems) * 2);
    w.pooled = (float*)p; p += align256(B * D * 4);
    w.rows = (int*)p;
    w.seg = w.rows + B;
    p += align256((2 * B + 1) * 4);
    w.part = (float*)p; p += align256(ce::kGemmPartElems * 4);
    w.stats = (float2*)p; p += align256(rows * 8);
    w.stats_part = (float2*)p;
    return w;
}

size_t vision_bytes(const ce_handle* h, long B) {
    const long Lv = (long)h->G * h->G + 1;
    return tower_bytes(B * Lv, h->cfg.vision.width, h->cfg.vision.mlp_width, B * h->G * h->G * h->Kp, B);
}
size_t text_bytes(const ce_handle* h, long B) {
    return tower_bytes(B * h->cfg.context_length, h->cfg.text.width, h->cfg.text.mlp_width, 0, B);
}

int grow_buffer(char*& buf, size_t& bytes, size_t need) {
    if (need <= bytes) return CE_OK;
    HIP_TRY(hipDeviceSynchronize());
    if (buf) HIP_TRY(hipFree(buf));
    buf = nullptr;
    bytes = 0;
    if (hipMalloc(&buf, need) != hipSuccess) {
        buf = nullptr;
        (void)hipGetLastError();
        return fail(CE_ERR_OOM, "cannot allocate %zu bytes of workspace", need);
    }
    bytes = need;
    return CE_OK;
}
int ensure_ws(ce_handle* h, size_t need) { return grow_buffer(h->ws, h->ws_bytes, need); }
int ensure_ws_text(ce_handle* h, size_t need) { return grow_buffer(h->ws_t, h->ws_t_bytes, need); }

int ensure_tmp(ce_handle* h, size_t need) {
    if (need <= h->tmp_bytes) return CE_OK;
    HIP_TRY(hipDeviceSynchronize());
    if (h->tmp) HIP_TRY(hipFree(h->tmp));
    h->tmp = nullptr;
    h->tmp_bytes = 0;
    if (hipMalloc(&h->tmp, need) != hipSuccess) {
        h->tmp = nullptr;
        (void)hipGetLastError();
        return fail(CE_ERR_OOM, "cannot allocate %zu bytes of scratch", need);
    }
    h->tmp_bytes = need;
    return CE_OK;
}

// ---------------------------------------------------------------------------------------------
// building blocks
struct EpiArgs {
    int epi = ce::EPI_PLAIN;
    bf16_t* xb = nullptr;
    float2* stats_part = nullptr;
    const float2* fold_stats = nullptr;
    const float* fold_c = nullptr;
    const bf16_t* rhl = nullptr;     // hi/lo residual planes (EPI_LN_STATS_HL / EPI_HL_F32)
    long hl_plane = 0;
    bool onetile = false;            // one tile per four-wave workgroup (the text tower's small grids)
    const int* m_dev = nullptr;      // packed rows: live row count on the device
    long ldo = 0;                    // output row stride (0: N)
};

int gemm(ce_handle* h, hipStream_t s, const char* tag, const bf16_t* A, long lda, const bf16_t* Wt,
         int M, int N, int K, const float* bias, int act, const float* resid, void* out, bool out_bf16,
         int grp = 0, int o_gs = 0, int o_go = 0, int r_gs = 0, int r_go = 0, const EpiArgs& ea = EpiArgs()) {
    ce::GemmParams p{};
    p.A = A; p.lda = lda; p.W = Wt; p.ldw = K;
    p.M = M; p.N = N; p.K = K;
    p.bias = bias;
    p.resid = resid; p.ldr = N;
    p.out = out; p.ldo = ea.ldo ? ea.ldo : N;
    p.grp = grp; p.o_gs = o_gs; p.o_go = o_go; p.r_gs = r_gs; p.r_go = r_go;
    p.part = h->cur_part;            // split-K tail slabs of the tower being run (null: no split)
    p.part_elems = h->cur_part ? ce::kGemmPartElems : 0;
    p.xb = ea.xb; p.stats_part = ea.stats_part; p.fold_stats = ea.fold_stats; p.fold_c = ea.fold_c;
    p.rhl = ea.rhl; p.hl_plane = ea.hl_plane;
    p.onetile = ea.onetile ? 1 : 0;
    p.m_dev = ea.m_dev;
    const double flops = 2.0 * M * N * K;
    // algorithmic bytes: A, W, the residual read (f32 or two bf16 planes: 4 B either way), the output
    // (f32, bf16, or two bf16 planes) and the bf16 copy of EPI_LN_STATS
    const bool hl = ea.epi == ce::EPI_LN_STATS_HL || ea.epi == ce::EPI_HL_F32;
    const double bytes = 2.0 * ((double)M * K + (double)N * K) + (double)M * N * (out_bf16 ? 2 : 4) +
                         ((resid || hl) ? (double)M * N * 4 : 0.0) +
                         (ea.xb && ea.epi == ce::EPI_LN_STATS ? (double)M * N * 2 : 0.0);
    // packed rows: the live count is on the device; a full profile pass has read it back (seg_host)
    double work = 1.0;
    if (ea.m_dev) {
        const bool known = h->seg_dev && ea.m_dev == h->seg_dev + (h->seg_host.size() - 1);
        work = known && M > 0 ? (double)h->seg_host.back() / M : 0.0;
    }
    return timed(h, s, tag, flops * work, bytes * work,
                 [&] { return ce::launch_gemm(p, act, out_bf16, s, ea.epi); });
}

int layernorm(ce_handle* h, hipStream_t s, const char* tag, const float* in, void* out, bool out_bf16,
              const float* w, const float* b, int rows, int D, int grp = 0, int i_gs = 0, int i_go = 0,
              int o_gs = 0, int o_go = 0, const float* w2 = nullptr, const float* b2 = nullptr,
              const float* rc = nullptr, const float* rs = nullptr, int rope_P = 1) {
    ce::LNParams p{};
    p.in = in; p.ldi = D; p.out = out; p.ldo = D;
    p.w = w; p.b = b; p.rows = rows; p.D = D;
    p.grp = grp; p.i_gs = i_gs; p.i_go = i_go; p.o_gs = o_gs; p.o_go = o_go;
    p.w2 = w2; p.b2 = b2; p.rope_cos = rc; p.rope_sin = rs; p.rope_P = rope_P;
    const double bytes = (double)rows * D * (4.0 + (out_bf16 ? 2.0 : 4.0));
    return timed(h, s, tag, 0.0, bytes, [&] { return ce::launch_layernorm(p, out_bf16, s); });
}

int act_code(const ce_handle* h) { return h->cfg.activation == CE_ACT_QUICK_GELU ? ce::ACT_QGELU_ : ce::ACT_GELU_; }

// one pre-LN residual block (transformer.py:257-268) on the f32 stream w.x [B*L][D]
int run_block(ce_handle* h, hipStream_t s, const TowerWs& w, const Blk& k, int B, int L, int D, int H,
              int F, bool causal, bool vis) {
    const int M = B * L;
    struct PartScope {      // split-K slabs of this tower for the block's GEMMs, cleared on every exit
        ce_handle* h;
        ~PartScope() { h->cur_part = nullptr; }
    } scope{h};
    h->cur_part = w.part;
    CE_TRY(layernorm(h, s, vis ? "ln_v" : "ln_t", w.x, w.xn, true, k.ln1w, k.ln1b, M, D));
    CE_TRY(gemm(h, s, vis ? "gemm_qkv_v" : "gemm_qkv_t", w.xn, D, k.wqkv, M, 3 * D, D, k.bqkv, ce::ACT_NONE_,
                nullptr, w.qkv, true));
    {
        // algorithmic attention work: QK^T and PV over the full L x L score matrix
        const double flops = 4.0 * B * H * (double)L * L * 64;
        const double bytes = (double)M * 3 * D * 2 + (double)M * D * 2;
        CE_TRY(timed(h, s, vis ? "attn_v" : "attn_t", flops, bytes,
                     [&] { return ce::launch_attention(w.qkv, w.att, B, L, H, causal, true, s); }));
    }
    CE_TRY(gemm(h, s, vis ? "gemm_out_v" : "gemm_out_t", w.att, D, k.wout, M, D, D, k.bout, ce::ACT_NONE_, w.x,
                w.x, false));
    CE_TRY(layernorm(h, s, vis ? "ln_v" : "ln_t", w.x, w.xn, true, k.ln2w, k.ln2b, M, D));
    CE_TRY(gemm(h, s, vis ? "gemm_fc_v" : "gemm_fc_t", w.xn, D, k.wfc, M, F, D, k.bfc, act_code(h), nullptr,
                w.hid, true));
    CE_TRY(gemm(h, s, vis ? "gemm_proj_v" : "gemm_proj_t", w.hid, F, k.wproj, M, D, F, k.bproj, ce::ACT_NONE_,
                w.x, w.x, false));
    return CE_OK;
}

int check_launch(hipError_t e, const char* what) {
    if (e != hipSuccess) return fail(CE_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    return CE_OK;
}

// folded weights of one vision block (fold_linear); null when the fold is not current
struct FoldBlk {
    const bf16_t *wqkv, *wfc;
    const float *cqkv, *dqkv, *cfc, *dfc;
};

bool fold_block(const ce_handle* h, const std::string& p, FoldBlk& f) {
    const std::string q = p + "attn.in_proj_weight", m = p + "mlp.c_fc.weight";
    auto ok = [&](const std::string& n) { auto it = h->folded.find(n); return it != h->folded.end() && it->second; };
    if (!ok(q) || !ok(m)) return false;
    f.wqkv = W<bf16_t>(h, q + "@fold"); f.cqkv = W(h, q + "@fold_c"); f.dqkv = W(h, q + "@fold_d");
    f.wfc = W<bf16_t>(h, m + "@fold"); f.cfc = W(h, m + "@fold_c"); f.dfc = W(h, m + "@fold_d");
    return f.wqkv && f.cqkv && f.dqkv && f.wfc && f.cfc && f.dfc;
}

// run_block with both pre-LNs folded into their GEMMs (either tower; the text tower's attention is
// causal).  On entry w.xn = bf16(w.x) (with the hi/lo stream: the hi plane, w.xlo the lo plane) and
// w.stats = (mu, rstd) of every row of w.x; the residual GEMMs re-establish both for the next block
// (the last block of the tower writes f32 w.x instead).
int run_block_folded(ce_handle* h, hipStream_t s, const TowerWs& w, const Blk& k, const FoldBlk& f, int B, int L,
                     int D, int H, int F, bool last, bool vis = true, const int* seg = nullptr) {
    const int M = B * L;
    struct PartScope {
        ce_handle* h;
        ~PartScope() { h->cur_part = nullptr; }
    } scope{h};
    h->cur_part = w.part;
    EpiArgs fold;
    fold.epi = ce::EPI_LN_FOLD;
    fold.fold_stats = w.stats;
    EpiArgs st;
    st.epi = ce::EPI_LN_STATS;
    st.xb = w.xn;
    st.stats_part = w.stats_part;
    // hi/lo stream: the residual GEMMs read and rewrite the planes (xn = hi, xlo = lo) in place of
    // the f32 x and its bf16 copy; the tower's last one writes f32 x for ln_post
    const bool hl = h->resid_hl;
    const float* resid = w.x;
    if (hl) {
        st.epi = ce::EPI_LN_STATS_HL;
        st.rhl = w.xn;
        st.hl_plane = (long)M * D;
        resid = nullptr;
    }
    EpiArgs last_ea;
    if (hl) {
        last_ea.epi = ce::EPI_HL_F32;
        last_ea.rhl = w.xn;
        last_ea.hl_plane = (long)M * D;
    }
    // the text tower's small grids run beside the image tower's persistent GEMMs (second stream):
    // four-wave kernel, one tile per workgroup, so they take CUs a tile at a time
    fold.onetile = st.onetile = last_ea.onetile = !vis;
    // packed text rows (pooled-only calls): seg[B] live rows of the B * L, sequences by seg
    const int* m_dev = seg ? seg + B : nullptr;
    fold.m_dev = st.m_dev = m_dev;
    auto finalize = [&] {
        return timed(h, s, vis ? "ln_stats_v" : "ln_stats_t", 0.0, (double)M * (D / 64) * 8 + (double)M * 8,
                     [&] { return ce::launch_ln_stats_finalize(w.stats, w.stats_part, M, D / 64, s, m_dev); });
    };
    fold.fold_c = f.cqkv;
    CE_TRY(gemm(h, s, vis ? "gemm_qkv_v" : "gemm_qkv_t", w.xn, D, f.wqkv, M, 3 * D, D, f.dqkv, ce::ACT_NONE_,
                nullptr, w.qkv, true, 0, 0, 0, 0, 0, fold));
    {
        double flops = 4.0 * B * H * (double)L * L * 64;
        double bytes = (double)M * 3 * D * 2 + (double)M * D * 2;
        if (seg) {
            // packed causal sequences of n_b = EOT + 1 rows: the full n_b x n_b score matrix each (as the
            // reference's count of a forward), when a profile pass has read the offsets back
            flops = bytes = 0.0;
            if (seg == h->seg_dev && (int)h->seg_host.size() == B + 1)
                for (int b = 0; b < B; ++b) {
                    const double n = h->seg_host[b + 1] - h->seg_host[b];
                    flops += 4.0 * H * n * n * 64;
                    bytes += n * (3 * D * 2 + D * 2);
                }
        }
        CE_TRY(timed(h, s, vis ? "attn_v" : "attn_t", flops, bytes,
                     [&] { return ce::launch_attention(w.qkv, w.att, B, L, H, !vis, true, s, nullptr, seg); }));
    }
    CE_TRY(gemm(h, s, vis ? "gemm_out_v" : "gemm_out_t", w.att, D, k.wout, M, D, D, k.bout, ce::ACT_NONE_, resid,
                w.x, false, 0, 0, 0, 0, 0, st));
    CE_TRY(finalize());
    fold.fold_c = f.cfc;
    CE_TRY(gemm(h, s, vis ? "gemm_fc_v" : "gemm_fc_t", w.xn, D, f.wfc, M, F, D, f.dfc, act_code(h), nullptr, w.hid,
                true, 0, 0, 0, 0, 0, fold));
    const char* tproj = vis ? "gemm_proj_v" : "gemm_proj_t";
    if (last) {
        CE_TRY(gemm(h, s, tproj, w.hid, F, k.wproj, M, D, F, k.bproj, ce::ACT_NONE_, resid, w.x, false,
                    0, 0, 0, 0, 0, last_ea));
    } else {
        CE_TRY(gemm(h, s, tproj, w.hid, F, k.wproj, M, D, F, k.bproj, ce::ACT_NONE_, resid, w.x, false,
                    0, 0, 0, 0, 0, st));
        CE_TRY(finalize());
    }
    return CE_OK;
}

// The last folded block of a tower when only its pooled rows are consumed (pooled-only
// encode_image / encode_text): row sel[b] of sequence b (null: b * L, the CLS row).  The QKV GEMM
// still covers every row (keys and values of the whole sequence); attention runs for the selected
// query rows only, and out-proj, c_fc and c_proj for those B rows — the other rows' outputs of
// this block feed nothing (the reference pools x[:, 0] / x[arange, argmax] after ln_post /
// ln_final, transformer.py:718-741, model.py:295-299).  Leaves the selected rows' final f32 x
// compact in w.x [B][D].  Compact work buffers: attention rows, then the residual hi/lo planes, in
// w.att; LN statistics of the B rows in w.stats / w.stats_part; c_fc output in w.hid.
int run_block_pooled(ce_handle* h, hipStream_t s, const TowerWs& w, const Blk& k, const FoldBlk& f, int B, int L,
                     int D, int H, int F, const int* sel, bool vis, const int* seg = nullptr) {
    const int M = B * L;
    struct PartScope {
        ce_handle* h;
        ~PartScope() { h->cur_part = nullptr; }
    } scope{h};
    h->cur_part = w.part;
    EpiArgs fold;
    fold.epi = ce::EPI_LN_FOLD;
    fold.fold_stats = w.stats;
    fold.onetile = !vis;
    fold.m_dev = seg ? seg + B : nullptr;
    // image tower: K and V of every row (in_proj rows D..3D into qkv's K | V thirds), the pooled
    // rows' q computed inside the attention kernel (the q third of 147,712 rows is 0.28 ms); text
    // tower (a few thousand packed rows): the whole QKV GEMM, cheaper than 64 W' rows per workgroup
    if (vis) {
        fold.fold_c = f.cqkv + D;
        fold.ldo = 3L * D;
        CE_TRY(gemm(h, s, "gemm_kv_pool_v", w.xn, D, f.wqkv + (size_t)D * D, M, 2 * D, D, f.dqkv + D, ce::ACT_NONE_,
                    nullptr, w.qkv + D, true, 0, 0, 0, 0, 0, fold));
        fold.ldo = 0;
    } else {
        fold.fold_c = f.cqkv;
        CE_TRY(gemm(h, s, "gemm_qkv_t", w.xn, D, f.wqkv, M, 3 * D, D, f.dqkv, ce::ACT_NONE_, nullptr, w.qkv, true,
                    0, 0, 0, 0, 0, fold));
    }
    bf16_t* att = w.att;                          // [B][D]
    bf16_t* xc = w.att + (size_t)B * D;           // hi plane [B][D], lo plane after it
    const long cplane = (long)B * D;
    {
        const double flops = 4.0 * B * H * (double)L * 64;
        const double bytes = (double)M * 2 * D * 2 + (double)B * D * 2 * 4;
        CE_TRY(timed(h, s, vis ? "attn_pool_v" : "attn_pool_t", flops, bytes, [&] {
            return ce::launch_attention_rows(w.qkv, sel, att, B, L, H, !vis, w.xn, (long)M * D, xc, cplane, s, seg,
                                             vis ? f.wqkv : nullptr, f.cqkv, f.dqkv, w.stats);
        }));
    }
    EpiArgs st;
    st.epi = ce::EPI_LN_STATS_HL;
    st.xb = xc;
    st.stats_part = w.stats_part;
    st.rhl = xc;
    st.hl_plane = cplane;
    CE_TRY(gemm(h, s, vis ? "gemm_out_pool_v" : "gemm_out_pool_t", att, D, k.wout, B, D, D, k.bout, ce::ACT_NONE_, nullptr,
                w.x, false, 0, 0, 0, 0, 0, st));
    CE_TRY(timed(h, s, vis ? "ln_stats_pool_v" : "ln_stats_pool_t", 0.0, (double)B * (D / 64) * 8 + (double)B * 8,
                 [&] { return ce::launch_ln_stats_finalize(w.stats, w.stats_part, B, D / 64, s); }));
    fold.fold_c = f.cfc;
    fold.m_dev = nullptr;
    CE_TRY(gemm(h, s, vis ? "gemm_fc_pool_v" : "gemm_fc_pool_t", xc, D, f.wfc, B, F, D, f.dfc, act_code(h), nullptr, w.hid,
                true, 0, 0, 0, 0, 0, fold));
    EpiArgs last_ea;
    last_ea.epi = ce::EPI_HL_F32;
    last_ea.rhl = xc;
    last_ea.hl_plane = cplane;
    return gemm(h, s, vis ? "gemm_proj_pool_v" : "gemm_proj_pool_t", w.hid, F, k.wproj, B, D, F, k.bproj, ce::ACT_NONE_,
                nullptr, w.x, false, 0, 0, 0, 0, 0, last_ea);
}

// Vision tower.  Leaves the final residual stream in w.x.  out_pooled may be null.
int run_vision(ce_handle* h, hipStream_t s, const TowerWs& w, const void* pix, bool pix_bf16, int B,
               float* out_pooled, bool normalize, bool keep_tokens = true) {
    const ce_config& c = h->cfg;
    const int D = c.vision.width, G = h->G, P = G * G, Lv = P + 1;
    // _embeds: conv1 as a patch GEMM whose epilogue scatters row (b,p) to b*Lv+1+p and adds pos[1+p]
    CE_TRY(timed(h, s, "im2col", 0.0, (double)B * 3 * c.image_size * c.image_size * (pix_bf16 ? 2 : 4) +
                                          (double)B * P * h->Kp * 2,
                 [&] { return ce::launch_im2col(pix, pix_bf16, w.hid, B, c.image_size, c.patch_size, h->Kp, s); }));
    CE_TRY(gemm(h, s, "gemm_patch", w.hid, h->Kp, W<bf16_t>(h, "visual.conv1.weight"), B * P, D, h->Kp, nullptr,
                ce::ACT_NONE_, W(h, "visual.positional_embedding"), w.x, false, P, Lv, 1, 0, 1));
    CE_TRY(check_launch(ce::launch_cls_rows(w.x, W(h, "visual.class_embedding"), W(h, "visual.positional_embedding"),
                                            B, Lv, D, s), "cls_rows"));
    // LN folding needs every block's fold current and D a multiple of 64 (the slab statistics)
    std::vector<FoldBlk> folds(c.vision.layers);
    bool use_fold = h->ln_fold && D % 64 == 0 && D / 64 <= 64;
    for (int i = 0; use_fold && i < c.vision.layers; ++i)
        use_fold = fold_block(h, "visual.transformer.resblocks." + std::to_string(i) + ".", folds[i]);
    if (use_fold) {
        // ln_pre in place, also emitting bf16(x) and the row statistics block 0's folded LN needs
        ce::LNParams p{};
        p.in = w.x; p.ldi = D; p.out = w.x; p.ldo = D;
        p.w = W(h, "visual.ln_pre.weight"); p.b = W(h, "visual.ln_pre.bias"); p.rows = B * Lv; p.D = D;
        p.xb = w.xn; p.stats = w.stats;
        if (h->resid_hl) p.xlo = w.xlo;
        CE_TRY(timed(h, s, "ln_v", 0.0, (double)B * Lv * D * (h->resid_hl ? 12.0 : 10.0),
                     [&] { return ce::launch_layernorm(p, false, s); }));
    } else {
        CE_TRY(layernorm(h, s, "ln_v", w.x, w.x, false, W(h, "visual.ln_pre.weight"), W(h, "visual.ln_pre.bias"),
                         B * Lv, D));
    }
    // pooled rows only (no tokens wanted): the last block for the CLS rows alone
    const bool prune = out_pooled && !keep_tokens && use_fold && h->resid_hl && h->pooled_prune && Lv >= 3;
    for (int i = 0; i < c.vision.layers; ++i) {
        const Blk k = block_ptrs(h, "visual.transformer.resblocks." + std::to_string(i) + ".");
        const bool last = i + 1 == c.vision.layers;
        if (prune && last)
            CE_TRY(run_block_pooled(h, s, w, k, folds[i], B, Lv, D, c.vision.heads, c.vision.mlp_width, nullptr,
                                    true));
        else if (use_fold)
            CE_TRY(run_block_folded(h, s, w, k, folds[i], B, Lv, D, c.vision.heads, c.vision.mlp_width, last));
        else
            CE_TRY(run_block(h, s, w, k, B, Lv, D, c.vision.heads, c.vision.mlp_width, false, true));
    }
    if (out_pooled) {
        CE_TRY(check_launch(ce::launch_ln_gather(w.pooled, w.x, nullptr, prune ? (long)D : (long)Lv * D, B, D,
                                                 W(h, "visual.ln_post.weight"), W(h, "visual.ln_post.bias"), s),
                            "ln_post(pool)"));
        ce::FGemmParams fp{};
        fp.A = w.pooled; fp.lda = D; fp.B = W(h, "visual.proj"); fp.ldb = c.embed_dim;
        fp.C = out_pooled; fp.ldc = c.embed_dim; fp.M = B; fp.N = c.embed_dim; fp.K = D; fp.batch = 1;
        fp.alpha = 1.f;
        CE_TRY(check_launch(ce::launch_fgemm(fp, false, s), "visual.proj"));
        if (normalize) CE_TRY(check_launch(ce::launch_l2norm(out_pooled, out_pooled, B, c.embed_dim, s), "normalize"));
    }
    return CE_OK;
}

int run_text(ce_handle* h, hipStream_t s, const TowerWs& w, const int64_t* ids, int B, float* out_pooled,
             bool normalize, bool keep_tokens = true) {
    const ce_config& c = h->cfg;
    const int D = c.text.width, L = c.context_length;
    // LN folding as in the image tower: every block's fold current, D a multiple of 64
    std::vector<FoldBlk> folds(c.text.layers);
    // (the embedding kernel that seeds the folded stream covers these widths; others run unfolded)
    const bool embed_ok = D == 256 || D == 512 || D == 768 || D == 1024 || D == 1280;
    bool use_fold = h->ln_fold && embed_ok && c.text.layers > 0;
    for (int i = 0; use_fold && i < c.text.layers; ++i)
        use_fold = fold_block(h, "transformer.resblocks." + std::to_string(i) + ".", folds[i]);
    // pooled rows only (no tokens wanted): the last block for the EOT rows alone, and every block on
    // the packed rows 0..EOT of each caption
    // packed rows need GEMM kernels that clip at the device row count: the default schedule's
    // (SCHED 1 and its four-wave / staged-residual kernels); a pinned other schedule runs every row
    const bool prune = out_pooled && !keep_tokens && use_fold && h->resid_hl && h->pooled_prune && L >= 3 &&
                       ce::current_gemm_sched() == 1;
    const int* seg = prune ? w.seg : nullptr;
    if (prune) CE_TRY(check_launch(ce::launch_text_pack(w.rows, w.seg, ids, B, L, s), "text_pack"));
    else if (out_pooled) CE_TRY(check_launch(ce::launch_argmax_rows(w.rows, ids, B, L, s), "argmax"));
    h->seg_dev = nullptr;
    h->seg_host.clear();
    if (prune && h->timing && h->timing_only.empty()) {
        // full profile pass (every launch bracketed, outside any timed region): read the packed
        // sequence offsets back once so the packed launches report their work
        h->seg_host.resize(B + 1);
        HIP_TRY(hipMemcpyAsync(h->seg_host.data(), w.seg, (B + 1) * sizeof(int), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        h->seg_dev = w.seg;
    }
    if (use_fold) {
        CE_TRY(timed(h, s, "t_embed", 0.0, (double)B * L * D * (h->resid_hl ? 12.0 : 10.0), [&] {
            return ce::launch_text_embed_stats(w.x, w.xn, h->resid_hl ? w.xlo : nullptr, w.stats, ids,
                                               W(h, "token_embedding.weight"), W(h, "positional_embedding"), B, L, D,
                                               c.vocab_size, s, seg);
        }));
    } else {
        CE_TRY(check_launch(ce::launch_text_embed(w.x, ids, W(h, "token_embedding.weight"),
                                                  W(h, "positional_embedding"), B, L, D, c.vocab_size, s),
                            "token_embedding"));
    }
    for (int i = 0; i < c.text.layers; ++i) {
        const Blk k = block_ptrs(h, "transformer.resblocks." + std::to_string(i) + ".");
        const bool last = i + 1 == c.text.layers;
        if (prune && last)
            CE_TRY(run_block_pooled(h, s, w, k, folds[i], B, L, D, c.text.heads, c.text.mlp_width, w.rows, false, seg));
        else if (use_fold)
            CE_TRY(run_block_folded(h, s, w, k, folds[i], B, L, D, c.text.heads, c.text.mlp_width, last, false, seg));
        else
            CE_TRY(run_block(h, s, w, k, B, L, D, c.text.heads, c.text.mlp_width, true, false));
    }
    if (out_pooled) {
        CE_TRY(check_launch(ce::launch_ln_gather(w.pooled, w.x, prune ? nullptr : w.rows, D, B, D, W(h, "ln_final.weight"),
                                                 W(h, "ln_final.bias"), s), "ln_final(pool)"));
        ce::FGemmParams fp{};
        fp.A = w.pooled; fp.lda = D; fp.B = W(h, "text_projection"); fp.ldb = c.embed_dim;
        fp.C = out_pooled; fp.ldc = c.embed_dim; fp.M = B; fp.N = c.embed_dim; fp.K = D; fp.batch = 1;
        fp.alpha = 1.f;
        CE_TRY(check_launch(ce::launch_fgemm(fp, false, s), "text_projection"));
        if (normalize) CE_TRY(check_launch(ce::launch_l2norm(out_pooled, out_pooled, B, c.embed_dim, s), "normalize"));
    }
    return CE_OK;
}

void host_rope_tables(int P, int D, std::vector<float>& cs, std::vector<float>& sn) {
    // mirrors apply_rope's f32 arithmetic: inv_freq = 1/(10000^(2i/D)); angle = pos * inv_freq
    const int half = D / 2;
    cs.resize((size_t)P * half);
    sn.resize((size_t)P * half);
    for (int i = 0; i < half; ++i) {
        const float expo = (float)(2 * i) / (float)D;
        const float inv = 1.0f / (float)pow(10000.0, (double)expo);   // see oracle.apply_rope
        for (int p = 0; p < P; ++p) {
            const float ang = (float)p * inv;
            cs[(size_t)p * half + i] = cosf(ang);
            sn[(size_t)p * half + i] = sinf(ang);
        }
    }
}

int upload(void** dst, const void* src, size_t bytes) {
    if (hipMalloc(dst, bytes) != hipSuccess) {
        (void)hipGetLastError();
        return fail(CE_ERR_OOM, "cannot allocate %zu bytes", bytes);
    }
    HIP_TRY(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
    return CE_OK;
}

bool valid_tower(const ce_tower_config& t) {
    return t.width > 0 && t.layers >= 0 && t.heads > 0 && t.width == t.heads * 64 && t.mlp_width > 0 &&
           t.width % 256 == 0 && t.width <= 1536 && t.mlp_width % 64 == 0;
}

// ---------------------------------------------------------------------------------------------
// Text-tower training: activations saved by the forward, scratch of the backward.  Per layer l:
// X[l] (block input, f32), XM[l] (after attention, f32), xn1/att/xn2 (bf16 [M][D]), qkv (bf16
// [M][3D]), pre/hh (c_fc pre-activation and activation, bf16 [M][F]); X[layers] feeds ln_final.
struct TrainWs {
    int B = 0, M = 0, Mp = 0, D = 0, F = 0, E = 0, nl = 0;
    std::vector<float*> X, XM;
    std::vector<bf16_t*> xn1, qkv, att, xn2, pre, hh;
    std::vector<float*> lse;     // [B][H][L] attention row log-sum-exp (log2 units) per layer
    int64_t* ids;
    int* rows;
    float *pooled, *u, *f;
    // backward scratch
    float *dres, *dxn, *dpool, *du, *pooledT, *colsum, *lnscr, *bpart;
    bf16_t *dres_b, *dA, *dB, *TA, *TB, *WT;
    float* part;
    void* emb;
    size_t emb_bytes;
};

size_t train_layout(const ce_handle* h, int B, TrainWs* w, char* base) {
    const ce_config& c = h->cfg;
    const int D = c.text.width, F = c.text.mlp_width, E = c.embed_dim, L = c.context_length, nl = c.text.layers;
    const long M = (long)B * L, Mp = (M + 63) / 64 * 64;
    const long NX = std::max(3L * D, (long)F);
    size_t off = 0;
    auto take = [&](size_t bytes) -> char* {
        char* r = base ? base + off : nullptr;
        off += align256(bytes);
        return r;
    };
    TrainWs t;
    t.B = B; t.M = (int)M; t.Mp = (int)Mp; t.D = D; t.F = F; t.E = E; t.nl = nl;
    for (int l = 0; l <= nl; ++l) t.X.push_back((float*)take(M * D * 4));
    for (int l = 0; l < nl; ++l) {
        t.XM.push_back((float*)take(M * D * 4));
        t.xn1.push_back((bf16_t*)take(M * D * 2));
        t.qkv.push_back((bf16_t*)take(M * 3 * D * 2));
        t.att.push_back((bf16_t*)take(M * D * 2));
        t.xn2.push_back((bf16_t*)take(M * D * 2));
        t.pre.push_back((bf16_t*)take(M * F * 2));
        t.hh.push_back((bf16_t*)take(M * F * 2));
        t.lse.push_back((float*)take(M * c.text.heads * 4));
    }
    t.ids = (int64_t*)take(M * 8);
    t.rows = (int*)take(B * 4);
    t.pooled = (float*)take((size_t)B * D * 4);
    t.u = (float*)take((size_t)B * E * 4);
    t.f = (float*)take((size_t)B * E * 4);
    t.dres = (float*)take(M * D * 4);
    t.dxn = (float*)take(M * D * 4);
    t.dpool = (float*)take((size_t)B * D * 4);
    t.du = (float*)take((size_t)B * E * 4);
    t.pooledT = (float*)take((size_t)B * D * 4);
    t.colsum = (float*)take(std::max({ce::colsum_scratch_floats((int)M, (int)NX), ce::act_bwd_colsum_scratch_floats((int)M, F),
                                      ce::colsum_scratch_floats((int)M, 3 * (int)D),
                                      ce::colsum_scratch_floats((int)B, 3 * (int)D)}) * 4);
    t.bpart = (float*)take((size_t)B * 3 * D * 4);      // attention backward: per-caption in_proj bias sums
    t.lnscr = (float*)take(ce::ln_bwd_scratch_floats((int)M, D) * 4);
    t.dres_b = (bf16_t*)take(M * D * 2);
    t.dA = (bf16_t*)take(M * NX * 2);
    t.dB = (bf16_t*)take(M * NX * 2);
    t.TA = (bf16_t*)take(NX * Mp * 2);
    t.TB = (bf16_t*)take(NX * Mp * 2);
    t.WT = (bf16_t*)take(NX * D * 2);
    t.part = (float*)take(ce::kGemmPartElems * 4);
    t.emb_bytes = ce::embed_bwd_scratch_bytes(B, L, D);
    t.emb = take(t.emb_bytes);
    if (w) *w = t;
    return off;
}

int train_ws(ce_handle* h, int B, TrainWs& w) {
    const size_t need = train_layout(h, B, nullptr, nullptr);
    CE_TRY(grow_buffer(h->tr, h->tr_bytes, need));
    train_layout(h, B, &w, h->tr);
    return CE_OK;
}

const char* kTextTrainable[] = {"ln_1.weight", "ln_1.bias", "attn.in_proj_weight", "attn.in_proj_bias",
                                "attn.out_proj.weight", "attn.out_proj.bias", "ln_2.weight", "ln_2.bias",
                                "mlp.c_fc.weight", "mlp.c_fc.bias", "mlp.c_proj.weight", "mlp.c_proj.bias"};

std::vector<std::string> text_trainable_names(const ce_handle* h) {
    std::vector<std::string> v = {"token_embedding.weight", "positional_embedding", "ln_final.weight",
                                  "ln_final.bias", "text_projection"};
    for (int l = 0; l < h->cfg.text.layers; ++l)
        for (const char* n : kTextTrainable) v.push_back("transformer.resblocks." + std::to_string(l) + "." + n);
    return v;
}

size_t spec_elems(const ce_handle* h, const std::string& n) {
    size_t c = 1;
    for (auto v : h->specs.at(n).shape) c *= (size_t)v;
    return c;
}

float* grad_of(ce_handle* h, const std::string& n) { return h->bound.at(n).second; }

int tgemm(ce_handle* h, hipStream_t s, const char* tag, const bf16_t* A, long lda, const bf16_t* Wt, long ldw, int M,
          int N, int K, const float* bias, int act, const float* resid, void* out, bool out_bf16, float* part) {
    ce::GemmParams p{};
    p.A = A; p.lda = lda; p.W = Wt; p.ldw = ldw;
    p.M = M; p.N = N; p.K = K;
    p.bias = bias;
    p.resid = resid; p.ldr = N;
    p.out = out; p.ldo = N;
    p.part = part;
    p.part_elems = part ? ce::kGemmPartElems : 0;
    return timed(h, s, tag, 2.0 * M * N * K, 0.0, [&] { return ce::launch_gemm(p, act, out_bf16, s); });
}

// activation backward in the dX_proj GEMM's epilogue (1, default) or as its own kernel (0)
std::atomic<int> g_act_bwd_fuse{ce::kKnobUnset};     // A/B knob (knobs.h)
int act_bwd_fuse_env() { return ce::env_int("CE_TRAIN_ACT_BWD_FUSE", 1) != 0; }
bool act_bwd_fuse() { return ce::knob_get(g_act_bwd_fuse, act_bwd_fuse_env) != 0; }

// weight gradients by the MN-major GEMM (gemm_tn.hip) or, 0, by transposed copies + the forward GEMM
std::atomic<int> g_dw_tn{ce::kKnobUnset};     // A/B knob (knobs.h)
int dw_tn_env() { return ce::env_int("CE_TRAIN_DW_TN", 1) != 0; }
bool dw_tn() { return ce::knob_get(g_dw_tn, dw_tn_env) != 0; }

// dW[M][N] = scale_m * sum over the T token rows of A[t][m] B[t][n]  (row-major activations in place)
int tgemm_tn(ce_handle* h, hipStream_t s, const char* tag, const bf16_t* A, long lda, const bf16_t* B, long ldb, int M,
             int N, int T, float* out, float* part, int scale_rows = 0, float scale = 1.f) {
    ce::TnParams p{};
    p.A = A; p.lda = lda; p.B = B; p.ldb = ldb;
    p.M = M; p.N = N; p.K = T;
    p.C = out; p.ldc = N;
    p.part = part; p.part_elems = part ? ce::kGemmPartElems : 0;
    p.scale_rows = scale_rows; p.scale = scale;
    return timed(h, s, tag, 2.0 * M * N * T, 0.0, [&] { return ce::launch_gemm_tn(p, s); });
}

// text forward keeping every activation the backward needs (open_clip encode_text, model.py:283-301)
int run_text_train(ce_handle* h, hipStream_t s, TrainWs& w, const int64_t* ids) {
    const ce_config& c = h->cfg;
    const int D = w.D, F = w.F, L = c.context_length, H = c.text.heads, M = w.M, B = w.B;
    HIP_TRY(hipMemcpyAsync(w.ids, ids, (size_t)M * 8, hipMemcpyDeviceToDevice, s));
    CE_TRY(timed(h, s, "t_token_embedding", 0.0, 0.0, [&] { return ce::launch_text_embed(w.X[0], w.ids, W(h, "token_embedding.weight"), W(h, "positional_embedding"),
                                              B, L, D, c.vocab_size, s); }));
    for (int l = 0; l < w.nl; ++l) {
        const Blk k = block_ptrs(h, "transformer.resblocks." + std::to_string(l) + ".");
        CE_TRY(layernorm(h, s, "ln_t", w.X[l], w.xn1[l], true, k.ln1w, k.ln1b, M, D));
        CE_TRY(tgemm(h, s, "train_qkv", w.xn1[l], D, k.wqkv, D, M, 3 * D, D, k.bqkv, ce::ACT_NONE_, nullptr, w.qkv[l],
                     true, w.part));
        CE_TRY(timed(h, s, "train_attn", 4.0 * B * H * (double)L * L * 64, 0.0,
                     [&] { return ce::launch_attention(w.qkv[l], w.att[l], B, L, H, true, true, s, w.lse[l]); }));
        CE_TRY(tgemm(h, s, "train_out", w.att[l], D, k.wout, D, M, D, D, k.bout, ce::ACT_NONE_, w.X[l], w.XM[l], false,
                     w.part));
        CE_TRY(layernorm(h, s, "ln_t", w.XM[l], w.xn2[l], true, k.ln2w, k.ln2b, M, D));
        {   // c_fc: the activation and the pre-activation copy the backward needs from one epilogue
            ce::GemmParams p{};
            p.A = w.xn2[l]; p.lda = D; p.W = k.wfc; p.ldw = D;
            p.M = M; p.N = F; p.K = D;
            p.bias = k.bfc;
            p.out = w.hh[l]; p.ldo = F;
            p.pre_out = w.pre[l];
            p.part = w.part; p.part_elems = ce::kGemmPartElems;
            CE_TRY(timed(h, s, "train_fc", 2.0 * M * F * D, 0.0, [&] { return ce::launch_gemm(p, act_code(h), true, s); }));
        }
        CE_TRY(tgemm(h, s, "train_proj", w.hh[l], F, k.wproj, F, M, D, F, k.bproj, ce::ACT_NONE_, w.XM[l], w.X[l + 1],
                     false, w.part));
    }
    CE_TRY(timed(h, s, "t_argmax", 0.0, 0.0, [&] { return ce::launch_argmax_rows(w.rows, w.ids, B, L, s); }));
    CE_TRY(timed(h, s, "t_ln_final_pool", 0.0, 0.0, [&] { return ce::launch_ln_gather(w.pooled, w.X[w.nl], w.rows, D, B, D, W(h, "ln_final.weight"),
                                             W(h, "ln_final.bias"), s); }));
    ce::FGemmParams fp{};
    fp.A = w.pooled; fp.lda = D; fp.B = W(h, "text_projection"); fp.ldb = w.E;
    fp.C = w.u; fp.ldc = w.E; fp.M = B; fp.N = w.E; fp.K = D; fp.batch = 1; fp.alpha = 1.f;
    CE_TRY(timed(h, s, "t_text_projection", 0.0, 0.0, [&] { return ce::launch_fgemm(fp, false, s); }));
    CE_TRY(timed(h, s, "t_normalize", 0.0, 0.0, [&] { return ce::launch_l2norm(w.f, w.u, B, w.E, s); }));
    return CE_OK;
}

// d(loss)/d(every bound text tensor) from d(loss)/d(normalised features) [B][E]
// events (optional, n_events = layers + 1; null entries skipped): events[0] is recorded once the head's
// gradients (ln_final, text_projection) are final, events[1 + i] once block layers - 1 - i's are, so a
// caller can all-reduce each bucket of blocks on another stream while the blocks below run (DDP's
// bucketed overlap, main.py:302); the embeddings' gradients are final when the stream reaches the end
int run_text_backward(ce_handle* h, hipStream_t s, TrainWs& w, const float* dfeat, void* const* events = nullptr,
                      int n_events = 0) {
    auto mark = [&](int i) -> int {
        if (events && i < n_events && events[i]) HIP_TRY(hipEventRecord((hipEvent_t)events[i], s));
        return CE_OK;
    };
    const ce_config& c = h->cfg;
    const int D = w.D, F = w.F, E = w.E, L = c.context_length, H = c.text.heads, M = w.M, Mp = w.Mp, B = w.B;
    const int act = act_code(h);
    // F.normalize, projection, ln_final on the EOT rows (transformer.py:839-855, model.py:300)
    CE_TRY(timed(h, s, "t_l2norm_bwd", 0.0, 0.0, [&] { return ce::launch_l2norm_bwd(w.du, w.u, dfeat, B, E, s); }));
    CE_TRY(timed(h, s, "t_transpose", 0.0, 0.0, [&] { return ce::launch_transpose_f32(w.pooledT, B, w.pooled, D, B, D, s); }));
    {
        ce::FGemmParams fp{};      // d text_projection [D][E] = pooled^T du
        fp.A = w.pooledT; fp.lda = B; fp.B = w.du; fp.ldb = E; fp.C = grad_of(h, "text_projection"); fp.ldc = E;
        fp.M = D; fp.N = E; fp.K = B; fp.batch = 1; fp.alpha = 1.f;
        CE_TRY(timed(h, s, "t_d_text_projection", 0.0, 0.0, [&] { return ce::launch_fgemm(fp, false, s); }));
        ce::FGemmParams fq{};      // d pooled [B][D] = du proj^T
        fq.A = w.du; fq.lda = E; fq.B = W(h, "text_projection"); fq.ldb = E; fq.C = w.dpool; fq.ldc = D;
        fq.M = B; fq.N = D; fq.K = E; fq.batch = 1; fq.alpha = 1.f;
        CE_TRY(timed(h, s, "t_d_pooled", 0.0, 0.0, [&] { return ce::launch_fgemm(fq, true, s); }));
    }
    HIP_TRY(hipMemsetAsync(w.dres, 0, (size_t)M * D * 4, s));
    HIP_TRY(hipMemsetAsync(w.dres_b, 0, (size_t)M * D * 2, s));
    // ln_final on the EOT rows; its dres rows are the top block's c_proj output gradient: the bf16 copy
    // and that bias's column sums come out of the same kernel
    const std::string top = "transformer.resblocks." + std::to_string(w.nl - 1) + ".";
    CE_TRY(timed(h, s, "t_ln_final_bwd", 0.0, 0.0, [&] { return ce::launch_ln_bwd(w.dres, w.X[w.nl], w.dpool, D, W(h, "ln_final.weight"), w.rows, B, D,
                                          grad_of(h, "ln_final.weight"), grad_of(h, "ln_final.bias"), false, false,
                                          w.lnscr, s, w.dres_b, grad_of(h, top + "mlp.c_proj.bias")); }));
    CE_TRY(mark(0));
    const float qs = ce::kAttnQScale;
    // MN-major dW GEMMs: widths that are multiples of 256 (ViT-B/L text towers: 512, 768) and
    // activations under the kernel's 32-bit DMA offsets (< 2 GB: up to ~340k token rows at F = 3072);
    // otherwise the transposed copies
    const bool tn = dw_tn() && D % 256 == 0 && F % 256 == 0 && (long)M * std::max(3 * D, F) * 2 <= 0x7fe00000L;
    bf16_t* const dxb = reinterpret_cast<bf16_t*>(w.dxn);     // [M][D] bf16 in the f32 buffer's space
    for (int l = w.nl - 1; l >= 0; --l) {
        const std::string pfx = "transformer.resblocks." + std::to_string(l) + ".";
        const Blk k = block_ptrs(h, pfx);
        auto G = [&](const char* n) { return grad_of(h, pfx + n); };
        // ---- MLP: X[l+1] = XM + c_proj(act(c_fc(ln_2 XM)))  (transformer.py:235-239, 267) ----
        // (dres_b and the c_proj bias gradient came out of the ln backward that produced dres)
        if (tn) {
            CE_TRY(tgemm_tn(h, s, "dW_proj", w.dres_b, D, w.hh[l], F, D, F, M, G("mlp.c_proj.weight"), w.part));
        } else {
            CE_TRY(timed(h, s, "t_transpose", 0.0, 0.0, [&] { return ce::launch_transpose_bf16(w.TA, Mp, w.dres, true, D, M, D, Mp, s); }));
            CE_TRY(timed(h, s, "t_transpose", 0.0, 0.0, [&] { return ce::launch_transpose_bf16(w.TB, Mp, w.hh[l], false, F, M, F, Mp, s); }));
            CE_TRY(tgemm(h, s, "dW_proj", w.TA, Mp, w.TB, Mp, D, F, Mp, nullptr, 0, nullptr, G("mlp.c_proj.weight"), false,
                         w.part));
        }
        CE_TRY(timed(h, s, "t_transpose", 0.0, 0.0, [&] { return ce::launch_transpose_bf16(w.WT, D, k.wproj, false, F, D, F, D, s); }));
        // dA = act'(pre) * (dres_b W_proj) and the c_fc bias gradient: one GEMM with the activation
        // backward and the bias column sums in its epilogue where the default four-wave kernel takes
        // this shape, else the GEMM then the activation-backward kernel (same values)
        ce::GemmParams pb{};
        pb.A = w.dres_b; pb.lda = D; pb.W = w.WT; pb.ldw = D;
        pb.M = M; pb.N = F; pb.K = D;
        pb.out = w.dA; pb.ldo = F;
        pb.bwd_pre = w.pre[l]; pb.bwd_part = w.colsum;
        if (act_bwd_fuse() && ce::gemm_act_bwd_fused(pb, act)) {
            CE_TRY(timed(h, s, "dX_proj_act", 2.0 * M * F * D, 0.0, [&] { return ce::launch_gemm_act_bwd(pb, act, s); }));
            CE_TRY(timed(h, s, "t_act_bwd", 0.0, 0.0, [&] {
                return ce::launch_colsum_finish(G("mlp.c_fc.bias"), w.colsum, (M + 127) / 128, F, s);
            }));
        } else {
            CE_TRY(tgemm(h, s, "dX_proj", w.dres_b, D, w.WT, D, M, F, D, nullptr, 0, nullptr, w.dA, true, w.part));
            CE_TRY(timed(h, s, "t_act_bwd", 0.0, 0.0, [&] {
                return ce::launch_act_bwd_colsum(w.dA, w.pre[l], w.dA, M, F, act, G("mlp.c_fc.bias"), w.colsum, s);
            }));
        }
        if (tn) {
            CE_TRY(tgemm_tn(h, s, "dW_fc", w.dA, F, w.xn2[l], D, F, D, M, G("mlp.c_fc.weight"), w.part));
        } else {
            CE_TRY(timed(h, s, "t_transpose", 0.0, 0.0, [&] { return ce::launch_transpose_bf16(w.TA, Mp, w.dA, false, F, M, F, Mp, s); }));
            CE_TRY(timed(h, s, "t_transpose", 0.0, 0.0, [&] { return ce::launch_transpose_bf16(w.TB, Mp, w.xn2[l], false, D, M, D, Mp, s); }));
            CE_TRY(tgemm(h, s, "dW_fc", w.TA, Mp, w.TB, Mp, F, D, Mp, nullptr, 0, nullptr, G("mlp.c_fc.weight"), false,
                         w.part));
        }
        CE_TRY(timed(h, s, "t_transpose", 0.0, 0.0, [&] { return ce::launch_transpose_bf16(w.WT, F, k.wfc, false, D, F, D, F, s); }));
        // (the LN-input gradients in bf16, as autocast's matmul gradients: half the bytes out of the dX
        // GEMMs and into the LN backward)
        CE_TRY(tgemm(h, s, "dX_fc", w.dA, F, w.WT, F, M, D, F, nullptr, 0, nullptr, dxb, true, w.part));
        CE_TRY(timed(h, s, "t_ln_2_bwd", 0.0, 0.0, [&] { return ce::launch_ln_bwd(w.dres, w.XM[l], nullptr, D, k.ln2w, nullptr, M, D, G("ln_2.weight"),
                                              G("ln_2.bias"), true, false, w.lnscr, s, w.dres_b,
                                              G("attn.out_proj.bias"), dxb); }));
        // ---- attention: XM = X + out_proj(MHA(ln_1 X))  (transformer.py:242-255, 266) ----
        if (tn) {
            CE_TRY(tgemm_tn(h, s, "dW_out", w.dres_b, D, w.att[l], D, D, D, M, G("attn.out_proj.weight"), w.part));
        } else {
            CE_TRY(timed(h, s, "t_transpose", 0.0, 0.0, [&] { return ce::launch_transpose_bf16(w.TA, Mp, w.dres, true, D, M, D, Mp, s); }));
            CE_TRY(timed(h, s, "t_transpose", 0.0, 0.0, [&] { return ce::launch_transpose_bf16(w.TB, Mp, w.att[l], false, D, M, D, Mp, s); }));
            CE_TRY(tgemm(h, s, "dW_out", w.TA, Mp, w.TB, Mp, D, D, Mp, nullptr, 0, nullptr, G("attn.out_proj.weight"),
                         false, w.part));
        }
        CE_TRY(timed(h, s, "t_transpose", 0.0, 0.0, [&] { return ce::launch_transpose_bf16(w.WT, D, k.wout, false, D, D, D, D, s); }));
        CE_TRY(tgemm(h, s, "dX_out", w.dres_b, D, w.WT, D, M, D, D, nullptr, 0, nullptr, w.dB, true, w.part));
        CE_TRY(timed(h, s, "attn_bwd", 10.0 * B * H * (double)L * L * 64, 0.0, [&] {
            return ce::launch_attention_bwd(w.dA, w.qkv[l], w.att[l], w.dB, w.lse[l], B, L, H, true, s,
                                            G("attn.in_proj_bias"), w.bpart, w.colsum);
        }));
        // in_proj: the engine's q rows carry kAttnQScale, so d(master q rows) = qs * d(engine q rows)
        CE_TRY(timed(h, s, "t_scale", 0.0, 0.0, [&] { return ce::launch_scale(G("attn.in_proj_bias"), D, qs, s); }));
        if (tn) {      // (the q rows' kAttnQScale applied by the split-K fixup)
            CE_TRY(tgemm_tn(h, s, "dW_qkv", w.dA, 3 * D, w.xn1[l], D, 3 * D, D, M, G("attn.in_proj_weight"), w.part, D,
                            qs));
        } else {
            CE_TRY(timed(h, s, "t_transpose", 0.0, 0.0, [&] { return ce::launch_transpose_bf16(w.TA, Mp, w.dA, false, 3 * D, M, 3 * D, Mp, s); }));
            CE_TRY(timed(h, s, "t_transpose", 0.0, 0.0, [&] { return ce::launch_transpose_bf16(w.TB, Mp, w.xn1[l], false, D, M, D, Mp, s); }));
            CE_TRY(tgemm(h, s, "dW_qkv", w.TA, Mp, w.TB, Mp, 3 * D, D, Mp, nullptr, 0, nullptr, G("attn.in_proj_weight"),
                         false, w.part));
            CE_TRY(timed(h, s, "t_scale", 0.0, 0.0, [&] { return ce::launch_scale(G("attn.in_proj_weight"), (long)D * D, qs, s); }));
        }
        CE_TRY(timed(h, s, "t_transpose", 0.0, 0.0, [&] { return ce::launch_transpose_bf16(w.WT, 3 * D, k.wqkv, false, D, 3 * D, D, 3 * D, s); }));
        CE_TRY(tgemm(h, s, "dX_qkv", w.dA, 3 * D, w.WT, 3 * D, M, D, 3 * D, nullptr, 0, nullptr, dxb, true, w.part));
        // (dres is now the gradient of X[l] = the c_proj output of block l - 1: its bf16 copy and that
        // bias's column sums come out of this kernel)
        float* below = l > 0 ? grad_of(h, "transformer.resblocks." + std::to_string(l - 1) + ".mlp.c_proj.bias") : nullptr;
        CE_TRY(timed(h, s, "t_ln_1_bwd", 0.0, 0.0, [&] { return ce::launch_ln_bwd(w.dres, w.X[l], nullptr, D, k.ln1w, nullptr, M, D, G("ln_1.weight"),
                                              G("ln_1.bias"), true, false, w.lnscr, s, w.dres_b, below, dxb); }));
        CE_TRY(mark(w.nl - l));
    }
    // token / positional embeddings (model.py:286-288)
    CE_TRY(timed(h, s, "t_embed_bwd", 0.0, 0.0, [&] { return ce::launch_embed_bwd(grad_of(h, "token_embedding.weight"), grad_of(h, "positional_embedding"),
                                             w.dres, w.ids, B, L, D, c.vocab_size, w.emb, w.emb_bytes, s); }));
    return CE_OK;
}

}  // namespace

// =============================================================================================
extern "C" {

const char* ce_last_error(void) { return g_err.c_str(); }

const char* ce_version(void) { return "clipembed 0.1.0 gfx950"; }

int ce_create(const ce_config* cfg, int device, ce_handle** out) {
    if (!cfg || !out) return fail(CE_ERR_INVALID, "ce_create: null argument");
    *out = nullptr;
    if (!valid_tower(cfg->vision) || !valid_tower(cfg->text))
        return fail(CE_ERR_INVALID, "ce_create: tower widths must be heads*64, multiple of 256 (got vision %d/%d, text %d/%d)",
                    cfg->vision.width, cfg->vision.heads, cfg->text.width, cfg->text.heads);
    if (cfg->patch_size <= 0 || cfg->image_size <= 0 || cfg->image_size % cfg->patch_size)
        return fail(CE_ERR_INVALID, "ce_create: image_size %d not a multiple of patch_size %d", cfg->image_size,
                    cfg->patch_size);
    if (cfg->embed_dim <= 0 || cfg->embed_dim % 64 || cfg->context_length <= 0 || cfg->vocab_size <= 0)
        return fail(CE_ERR_INVALID, "ce_create: bad embed_dim/context_length/vocab_size");
    if (cfg->activation != CE_ACT_GELU_ERF && cfg->activation != CE_ACT_QUICK_GELU)
        return fail(CE_ERR_INVALID, "ce_create: unknown activation %d", cfg->activation);
    if (cfg->pacl_dim < 0 || cfg->pacl_dim % 128 || cfg->pacl_dim > 1024)
        return fail(CE_ERR_INVALID, "ce_create: pacl_dim must be 0 or a multiple of 128 <= 1024");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        return fail(CE_ERR_HIP, "ce_create: no HIP device available");
    }
    if (device < 0 || device >= ndev) return fail(CE_ERR_INVALID, "ce_create: device %d out of range (%d)", device, ndev);
    DeviceGuard g(device);
    ce_handle* h = new ce_handle();
    if (const char* e = getenv("CE_LN_FOLD")) h->ln_fold = atoi(e) != 0;
    if (const char* e = getenv("CE_RESID_HL")) h->resid_hl = atoi(e) != 0;
    if (const char* e = getenv("CE_POOLED_PRUNE")) h->pooled_prune = atoi(e) != 0;
    h->cfg = *cfg;
    h->device = device;
    h->G = cfg->image_size / cfg->patch_size;
    h->Kp = ((3 * cfg->patch_size * cfg->patch_size) + 63) / 64 * 64;
    build_specs(h);
    if (hipMalloc(&h->scratch, 256) != hipSuccess) {
        delete h;
        return fail(CE_ERR_OOM, "ce_create: scratch allocation failed");
    }
    std::vector<float> cs, sn;
    const int P = h->G * h->G;
    host_rope_tables(P, cfg->vision.width, cs, sn);
    int rc = upload((void**)&h->rc_v, cs.data(), cs.size() * 4);
    if (rc == CE_OK) rc = upload((void**)&h->rs_v, sn.data(), sn.size() * 4);
    if (rc == CE_OK && cfg->pacl_dim > 0) {
        host_rope_tables(P, cfg->pacl_dim, cs, sn);
        rc = upload((void**)&h->rc_p, cs.data(), cs.size() * 4);
        if (rc == CE_OK) rc = upload((void**)&h->rs_p, sn.data(), sn.size() * 4);
    }
    if (rc != CE_OK) {
        ce_destroy(h);
        return rc;
    }
    *out = h;
    return CE_OK;
}

int ce_destroy(ce_handle* h) {
    if (!h) return CE_OK;
    DeviceGuard g(h->device);
    (void)hipDeviceSynchronize();
    for (auto& kv : h->dptr) (void)hipFree(kv.second);
    if (h->ws) (void)hipFree(h->ws);
    if (h->ws_t) (void)hipFree(h->ws_t);
    if (h->tmp) (void)hipFree(h->tmp);
    if (h->pool) (void)hipFree(h->pool);
    if (h->tr) (void)hipFree(h->tr);
    if (h->sp) (void)hipFree(h->sp);
    if (h->scratch) (void)hipFree(h->scratch);
    if (h->prep_host) (void)hipHostFree(h->prep_host);
    if (h->prep_dev) (void)hipFree(h->prep_dev);
    if (h->prep_tmp) (void)hipFree(h->prep_tmp);
    if (h->prep_ev) (void)hipEventDestroy(h->prep_ev);
    for (float* p : {h->rc_v, h->rs_v, h->rc_p, h->rs_p})
        if (p) (void)hipFree(p);
    for (auto& p : h->pending) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
    for (auto e : h->free_ev) (void)hipEventDestroy(e);
    delete h;
    return CE_OK;
}

namespace {

int tensor_f32(const ce_tensor& t, size_t cnt, std::vector<float>& f) {
    f.resize(cnt);
    switch (t.dtype) {
        case CE_F32: memcpy(f.data(), t.data, cnt * 4); return CE_OK;
        case CE_BF16: {
            const uint16_t* s = (const uint16_t*)t.data;
            for (size_t j = 0; j < cnt; ++j) f[j] = host_bf2f(s[j]);
            return CE_OK;
        }
        case CE_F16: {
            const uint16_t* s = (const uint16_t*)t.data;
            for (size_t j = 0; j < cnt; ++j) f[j] = host_h2f(s[j]);
            return CE_OK;
        }
        default: return fail(CE_ERR_INVALID, "ce_load_weights: '%s' unsupported dtype %d", t.name, t.dtype);
    }
}

int upload_named(ce_handle* h, const std::string& name, const void* src, size_t bytes) {
    void*& dp = h->dptr[name];
    if (!dp) {
        if (hipMalloc(&dp, bytes) != hipSuccess) {
            dp = nullptr;
            h->dptr.erase(name);
            (void)hipGetLastError();
            return fail(CE_ERR_OOM, "ce_load_weights: cannot allocate '%s'", name.c_str());
        }
    }
    HIP_TRY(hipMemcpy(dp, src, bytes, hipMemcpyHostToDevice));
    return CE_OK;
}

// LayerNorm folding.  The pre-LN of a block feeds exactly one GEMM, so
//   Linear(LN(x))_n = s_n * (sum_k W_nk (gamma_k (x_k - mu) rstd + beta_k) + b_n)
//                   = rstd * (sum_k W'_nk x_k - mu * c_n) + d_n
// with W'_nk = bf16(s_n gamma_k W_nk), c_n = sum_k W'_nk (of the rounded values, so the mean
// cancels exactly against the bf16 x the GEMM sees) and d_n = s_n (b_n + sum_k beta_k W_nk);
// s_n = kAttnQScale on the q rows of in_proj, else 1.  Only when all four source tensors come in
// one call is the fold recomputed; a partial update of any of them invalidates it.
int fold_linear(ce_handle* h, const ce_tensor* t, const std::map<std::string, int>& idx, const std::string& wn,
                const std::string& bn, const std::string& gn, const std::string& en, bool qrows) {
    auto find = [&](const std::string& k) { auto it = idx.find(k); return it == idx.end() ? -1 : it->second; };
    const int iw = find(wn), ib = find(bn), ig = find(gn), ie = find(en);
    if (iw < 0 && ib < 0 && ig < 0 && ie < 0) return CE_OK;
    if (iw < 0 || ib < 0 || ig < 0 || ie < 0) {
        h->folded[wn] = false;
        return CE_OK;
    }
    const std::vector<int64_t>& shp = h->specs.at(wn).shape;
    const size_t N = (size_t)shp[0], K = (size_t)shp[1];
    std::vector<float> W, b, g, e;
    CE_TRY(tensor_f32(t[iw], N * K, W));
    CE_TRY(tensor_f32(t[ib], N, b));
    CE_TRY(tensor_f32(t[ig], K, g));
    CE_TRY(tensor_f32(t[ie], K, e));
    std::vector<uint16_t> wf(N * K);
    std::vector<float> c(N), d(N);
    const size_t nq = qrows ? N / 3 : 0;
    for (size_t n = 0; n < N; ++n) {
        const float sn = n < nq ? ce::kAttnQScale : 1.f;
        double cs = 0.0, ds = 0.0;
        for (size_t k = 0; k < K; ++k) {
            const uint16_t v = host_f2bf(sn * (g[k] * W[n * K + k]));
            wf[n * K + k] = v;
            cs += host_bf2f(v);
            ds += (double)e[k] * W[n * K + k];
        }
        c[n] = (float)cs;
        d[n] = (float)((double)sn * ((double)b[n] + ds));
    }
    CE_TRY(upload_named(h, wn + "@fold", wf.data(), wf.size() * 2));
    CE_TRY(upload_named(h, wn + "@fold_c", c.data(), N * 4));
    CE_TRY(upload_named(h, wn + "@fold_d", d.data(), N * 4));
    h->folded[wn] = true;
    return CE_OK;
}

}  // namespace

int ce_load_weights(ce_handle* h, const ce_tensor* t, int n, int allow_unknown) {
    if (!h || (n > 0 && !t)) return fail(CE_ERR_INVALID, "ce_load_weights: null argument");
    DeviceGuard g(h->device);
    std::vector<float> f;
    std::map<std::string, int> idx;   // canonical name -> index in t, for the LN folds below
    for (int i = 0; i < n; ++i) {
        if (!t[i].name) return fail(CE_ERR_INVALID, "ce_load_weights: tensor %d has no name", i);
        const std::string name = canonical(h, t[i].name);
        auto it = h->specs.find(name);
        if (it == h->specs.end()) {
            if (allow_unknown) continue;
            return fail(CE_ERR_INVALID, "ce_load_weights: unknown weight '%s'", t[i].name);
        }
        const WSpec& sp = it->second;
        // shape check
        bool ok;
        if (sp.st == ST_SCALAR) {
            ok = t[i].ndim == 0 || (t[i].ndim == 1 && t[i].shape[0] == 1);
        } else {
            ok = t[i].ndim == (int)sp.shape.size();
            for (int d = 0; ok && d < t[i].ndim; ++d) ok = t[i].shape[d] == sp.shape[d];
        }
        if (!ok) {
            std::string got, want;
            for (int d = 0; d < t[i].ndim && d < 4; ++d) got += std::to_string(t[i].shape[d]) + ",";
            for (auto v : sp.shape) want += std::to_string(v) + ",";
            return fail(CE_ERR_INVALID, "ce_load_weights: '%s' has shape [%s] expected [%s]", t[i].name,
                        got.c_str(), want.c_str());
        }
        if (!t[i].data) return fail(CE_ERR_INVALID, "ce_load_weights: '%s' has no data", t[i].name);
        size_t cnt = 1;
        for (auto v : sp.shape) cnt *= (size_t)v;
        CE_TRY(tensor_f32(t[i], cnt, f));
        idx[name] = i;
        // Fold the attention score scale log2(e)/sqrt(head_dim) into the q rows of in_proj (the
        // first third of weight and bias): the attention kernel then works in log2 units with no
        // per-score multiply (attention.hip).  The host-side state dict keeps the original values.
        if (name.size() > 19 && (name.compare(name.size() - 19, 19, "attn.in_proj_weight") == 0 ||
                                 name.compare(name.size() - 17, 17, "attn.in_proj_bias") == 0)) {
            for (size_t j = 0; j < cnt / 3; ++j) f[j] *= ce::kAttnQScale;
        }
        std::vector<char> bytes;
        switch (sp.st) {
            case ST_SCALAR:
                h->logit_scale = f[0];
                h->loaded[name] = true;
                continue;
            case ST_F32:
                bytes.resize(cnt * 4);
                memcpy(bytes.data(), f.data(), cnt * 4);
                break;
            case ST_BF16: {
                bytes.resize(cnt * 2);
                uint16_t* o = (uint16_t*)bytes.data();
                for (size_t j = 0; j < cnt; ++j) o[j] = host_f2bf(f[j]);
                break;
            }
            case ST_BF16_PADK: {
                const size_t N = (size_t)sp.shape[0], K = cnt / N, Kp = (size_t)h->Kp;
                bytes.assign(N * Kp * 2, 0);
                uint16_t* o = (uint16_t*)bytes.data();
                for (size_t r = 0; r < N; ++r)
                    for (size_t k = 0; k < K; ++k) o[r * Kp + k] = host_f2bf(f[r * K + k]);
                break;
            }
            case ST_F32_T: {
                const size_t R = (size_t)sp.shape[0], C = (size_t)sp.shape[1];
                bytes.resize(cnt * 4);
                float* o = (float*)bytes.data();
                for (size_t r = 0; r < R; ++r)
                    for (size_t c = 0; c < C; ++c) o[c * R + r] = f[r * C + c];
                break;
            }
        }
        CE_TRY(upload_named(h, name, bytes.data(), bytes.size()));
        h->loaded[name] = true;
    }
    // LN folds of both towers' blocks
    std::vector<std::string> blocks;
    for (int l = 0; l < h->cfg.vision.layers; ++l) blocks.push_back("visual.transformer.resblocks." + std::to_string(l) + ".");
    for (int l = 0; l < h->cfg.text.layers; ++l) blocks.push_back("transformer.resblocks." + std::to_string(l) + ".");
    for (const std::string& P : blocks) {
        CE_TRY(fold_linear(h, t, idx, P + "attn.in_proj_weight", P + "attn.in_proj_bias", P + "ln_1.weight",
                           P + "ln_1.bias", true));
        CE_TRY(fold_linear(h, t, idx, P + "mlp.c_fc.weight", P + "mlp.c_fc.bias", P + "ln_2.weight",
                           P + "ln_2.bias", false));
    }
    return CE_OK;
}

int ce_missing_weights(ce_handle* h, int* n_missing, const char** first_missing) {
    if (!h) return fail(CE_ERR_INVALID, "ce_missing_weights: null handle");
    int n = 0;
    const char* first = nullptr;
    for (auto& kv : h->specs)
        if (kv.second.required && !h->loaded[kv.first]) {
            if (!first) first = kv.first.c_str();
            ++n;
        }
    if (n_missing) *n_missing = n;
    if (first_missing) *first_missing = first ? first : "";
    return CE_OK;
}

int ce_reserve(ce_handle* h, int max_images, int max_texts) {
    if (!h || max_images < 0 || max_texts < 0) return fail(CE_ERR_INVALID, "ce_reserve: bad argument");
    DeviceGuard g(h->device);
    CE_TRY(ensure_ws(h, std::max(vision_bytes(h, max_images), text_bytes(h, max_texts))));
    return ensure_ws_text(h, text_bytes(h, max_texts));
}

int ce_encode_image(ce_handle* h, void* stream, const void* pixels, int pixel_dtype, int B, int normalize,
                    float* out_pooled, void* out_tokens, int tokens_dtype) {
    if (!h) return fail(CE_ERR_INVALID, "ce_encode_image: null handle");
    if (B <= 0) return fail(CE_ERR_INVALID, "ce_encode_image: batch must be positive (got %d)", B);
    if (!pixels || (!out_pooled && !out_tokens)) return fail(CE_ERR_INVALID, "ce_encode_image: null buffer");
    if (pixel_dtype != CE_F32 && pixel_dtype != CE_BF16)
        return fail(CE_ERR_INVALID, "ce_encode_image: pixels must be f32 or bf16");
    if (out_tokens && tokens_dtype != CE_F32 && tokens_dtype != CE_BF16)
        return fail(CE_ERR_INVALID, "ce_encode_image: tokens must be f32 or bf16");
    CE_TRY(check_ready(h, false));
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    CE_TRY(ensure_ws(h, vision_bytes(h, B)));
    const long P = (long)h->G * h->G, Lv = P + 1;
    const int D = h->cfg.vision.width;
    TowerWs w = carve(h->ws, B * Lv, D, h->cfg.vision.mlp_width, B * P * h->Kp, B);
    CE_TRY(run_vision(h, s, w, pixels, pixel_dtype == CE_BF16, B, out_pooled, normalize != 0, out_tokens != nullptr));
    if (out_tokens)
        CE_TRY(layernorm(h, s, "ln_v", w.x, out_tokens, tokens_dtype == CE_BF16, W(h, "visual.ln_post.weight"),
                         W(h, "visual.ln_post.bias"), (int)(B * P), D, (int)P, (int)Lv, 1, (int)P, 0));
    return CE_OK;
}

int ce_encode_text(ce_handle* h, void* stream, const int64_t* ids, int B, int ctx, int normalize,
                   float* out_pooled, void* out_tokens, int tokens_dtype) {
    if (!h) return fail(CE_ERR_INVALID, "ce_encode_text: null handle");
    if (B <= 0) return fail(CE_ERR_INVALID, "ce_encode_text: batch must be positive (got %d)", B);
    if (ctx != h->cfg.context_length)
        return fail(CE_ERR_INVALID, "ce_encode_text: context length %d != %d", ctx, h->cfg.context_length);
    if (!ids || (!out_pooled && !out_tokens)) return fail(CE_ERR_INVALID, "ce_encode_text: null buffer");
    if (out_tokens && tokens_dtype != CE_F32 && tokens_dtype != CE_BF16)
        return fail(CE_ERR_INVALID, "ce_encode_text: tokens must be f32 or bf16");
    CE_TRY(check_ready(h, false));
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    CE_TRY(ensure_ws_text(h, text_bytes(h, B)));
    const int D = h->cfg.text.width;
    TowerWs w = carve(h->ws_t, (long)B * ctx, D, h->cfg.text.mlp_width, 0, B);
    CE_TRY(run_text(h, s, w, ids, B, out_pooled, normalize != 0, out_tokens != nullptr));
    if (out_tokens)
        CE_TRY(layernorm(h, s, "ln_final_t", w.x, out_tokens, tokens_dtype == CE_BF16, W(h, "ln_final.weight"),
                         W(h, "ln_final.bias"), B * ctx, D));
    return CE_OK;
}

int ce_get_logits(ce_handle* h, void* stream, const float* img, int Bi, const float* txt, int Bt, int D,
                  float scale, int normalize, float* out_image_logits, float* out_text_logits) {
    if (!h) return fail(CE_ERR_INVALID, "ce_get_logits: null handle");
    if (Bi <= 0 || Bt <= 0 || D <= 0) return fail(CE_ERR_INVALID, "ce_get_logits: bad sizes %d %d %d", Bi, Bt, D);
    if (!img || !txt || !out_image_logits) return fail(CE_ERR_INVALID, "ce_get_logits: null buffer");
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    const float* a = img;
    const float* b = txt;
    if (normalize) {
        CE_TRY(ensure_tmp(h, ((size_t)Bi + Bt) * D * 4));
        float* an = (float*)h->tmp;
        float* bn = an + (size_t)Bi * D;
        CE_TRY(check_launch(ce::launch_l2norm(an, img, Bi, D, s), "normalize"));
        CE_TRY(check_launch(ce::launch_l2norm(bn, txt, Bt, D, s), "normalize"));
        a = an;
        b = bn;
    }
    ce::FGemmParams fp{};
    fp.A = a; fp.lda = D; fp.B = b; fp.ldb = D; fp.C = out_image_logits; fp.ldc = Bt;
    fp.M = Bi; fp.N = Bt; fp.K = D; fp.batch = 1; fp.alpha = scale;
    fp.Ct = out_text_logits; fp.ldct = Bi;
    return timed(h, s, "logits", 2.0 * Bi * Bt * D, 4.0 * ((double)Bi * D + (double)Bt * D + (double)Bi * Bt),
                 [&] { return ce::launch_fgemm(fp, true, s); });
}

int ce_cross_entropy(ce_handle* h, void* stream, const float* logits, int R, int C, const int64_t* labels,
                     float* out_loss) {
    if (!h || !logits || !labels || !out_loss) return fail(CE_ERR_INVALID, "ce_cross_entropy: null argument");
    if (R <= 0 || C <= 0) return fail(CE_ERR_INVALID, "ce_cross_entropy: bad sizes");
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipMemsetAsync(h->scratch, 0, 16, s));
    CE_TRY(check_launch(ce::launch_cross_entropy_rows(h->scratch, logits, R, C, labels, s), "cross_entropy"));
    CE_TRY(check_launch(ce::launch_cross_entropy_finish(out_loss, h->scratch, s), "cross_entropy"));
    return CE_OK;
}

int ce_pacl_project_patches(ce_handle* h, void* stream, const void* tokens, int tokens_dtype, int B, int P,
                            int rope, void* out_proj, int out_dtype) {
    if (!h || !tokens || !out_proj) return fail(CE_ERR_INVALID, "ce_pacl_project_patches: null argument");
    if (h->cfg.pacl_dim <= 0) return fail(CE_ERR_STATE, "ce_pacl_project_patches: handle has no PACL head");
    if (tokens_dtype != CE_F32) return fail(CE_ERR_INVALID, "ce_pacl_project_patches: tokens must be f32");
    if (out_dtype != CE_F32 && out_dtype != CE_BF16) return fail(CE_ERR_INVALID, "ce_pacl_project_patches: out dtype");
    if (rope != CE_ROPE_NONE && rope != CE_ROPE_BEFORE)
        return fail(CE_ERR_INVALID, "ce_pacl_project_patches: rope must be NONE or BEFORE");
    if (B <= 0 || P <= 0) return fail(CE_ERR_INVALID, "ce_pacl_project_patches: bad sizes");
    if (rope == CE_ROPE_BEFORE && P != h->G * h->G)
        return fail(CE_ERR_INVALID, "ce_pacl_project_patches: rope tables cover %d patches", h->G * h->G);
    CE_TRY(check_ready(h, true));
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    const int Dv = h->cfg.vision.width, Pd = h->cfg.pacl_dim;
    const long M = (long)B * P;
    // scratch: [rope f32 M*Dv] | xn bf16 M*Dv | lin f32 M*Pd | h1 bf16 M*Pd
    const size_t need = align256(rope ? M * Dv * 4 : 0) + align256(M * Dv * 2) + align256(M * Pd * 4) + align256(M * Pd * 2);
    CE_TRY(ensure_ws(h, need));
    char* p = h->ws;
    float* rot = (float*)p; p += align256(rope ? M * Dv * 4 : 0);
    bf16_t* xn = (bf16_t*)p; p += align256(M * Dv * 2);
    float* lin = (float*)p; p += align256(M * Pd * 4);
    bf16_t* h1 = (bf16_t*)p;
    const float* src = (const float*)tokens;
    if (rope) {
        CE_TRY(check_launch(ce::launch_rope(rot, src, B, P, Dv, h->rc_v, h->rs_v, s), "apply_rope"));
        src = rot;
    }
    CE_TRY(layernorm(h, s, "ln_pacl", src, xn, true, W(h, "visual_projection.0.weight"), W(h, "visual_projection.0.bias"),
                     (int)M, Dv));
    CE_TRY(gemm(h, s, "gemm_pacl", xn, Dv, W<bf16_t>(h, "visual_projection.2.linear_projection.0.weight"), (int)M, Pd,
                Dv, W(h, "visual_projection.2.linear_projection.0.bias"), ce::ACT_NONE_, nullptr, lin, false));
    CE_TRY(gemm(h, s, "gemm_pacl", xn, Dv, W<bf16_t>(h, "visual_projection.2.non_linear_projection.0.weight"), (int)M,
                Pd, Dv, W(h, "visual_projection.2.non_linear_projection.0.bias"), ce::ACT_GELU_, nullptr, h1, true));
    CE_TRY(gemm(h, s, "gemm_pacl", h1, Pd, W<bf16_t>(h, "visual_projection.2.non_linear_projection.2.weight"), (int)M,
                Pd, Pd, W(h, "visual_projection.2.non_linear_projection.2.bias"), ce::ACT_NONE_, lin, out_proj,
                out_dtype == CE_BF16));
    return CE_OK;
}

int ce_pacl_project_text(ce_handle* h, void* stream, const float* text_pooled, int B, float* out_proj) {
    if (!h || !text_pooled || !out_proj) return fail(CE_ERR_INVALID, "ce_pacl_project_text: null argument");
    if (h->cfg.pacl_dim <= 0) return fail(CE_ERR_STATE, "ce_pacl_project_text: handle has no PACL head");
    if (B <= 0) return fail(CE_ERR_INVALID, "ce_pacl_project_text: bad batch");
    CE_TRY(check_ready(h, true));
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    const int E = h->cfg.embed_dim, Pd = h->cfg.pacl_dim;
    CE_TRY(ensure_tmp(h, (size_t)B * E * 4));
    float* ln = (float*)h->tmp;
    CE_TRY(check_launch(ce::launch_ln_gather(ln, text_pooled, nullptr, E, B, E, W(h, "text_projection.0.weight"),
                                             W(h, "text_projection.0.bias"), s), "pacl text ln"));
    ce::FGemmParams fp{};
    fp.A = ln; fp.lda = E; fp.B = W(h, "text_projection.2.weight"); fp.ldb = Pd; fp.C = out_proj; fp.ldc = Pd;
    fp.M = B; fp.N = Pd; fp.K = E; fp.batch = 1; fp.alpha = 1.f; fp.bias = W(h, "text_projection.2.bias");
    CE_TRY(check_launch(ce::launch_fgemm(fp, false, s), "pacl text linear"));
    return CE_OK;
}

int ce_pacl_pool(ce_handle* h, void* stream, const void* visual_proj, int vp_dtype, int Bi, int P,
                 const float* text_proj, int Bt, int Dp, int weight_mode, int rope_after, float* out_img,
                 float* out_txt) {
    if (!h || !visual_proj || !text_proj || !out_img) return fail(CE_ERR_INVALID, "ce_pacl_pool: null argument");
    if (Bi <= 0 || Bt <= 0 || P <= 0) return fail(CE_ERR_INVALID, "ce_pacl_pool: bad sizes");
    if (!(Bi == Bt || Bi == 1 || Bt == 1))
        return fail(CE_ERR_INVALID, "ce_pacl_pool: cannot broadcast %d images against %d texts", Bi, Bt);
    if (vp_dtype != CE_F32 && vp_dtype != CE_BF16) return fail(CE_ERR_INVALID, "ce_pacl_pool: visual_proj dtype");
    if (weight_mode != CE_PACL_ONES && weight_mode != CE_PACL_SIGMOID10)
        return fail(CE_ERR_INVALID, "ce_pacl_pool: unknown weight mode %d", weight_mode);
    if (rope_after && weight_mode != CE_PACL_SIGMOID10)
        return fail(CE_ERR_INVALID, "ce_pacl_pool: rope_after only affects the sigmoid10 activations");
    if (Dp % 128 || Dp > 1024) return fail(CE_ERR_INVALID, "ce_pacl_pool: Dp must be a multiple of 128 <= 1024");
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    const float *rc = nullptr, *rs = nullptr;
    std::vector<float> cs, sn;
    if (rope_after) {
        if (Dp == h->cfg.pacl_dim && P == h->G * h->G && h->rc_p) { rc = h->rc_p; rs = h->rs_p; }
        else if (Dp == h->cfg.vision.width && P == h->G * h->G) { rc = h->rc_v; rs = h->rs_v; }
        else return fail(CE_ERR_INVALID, "ce_pacl_pool: no RoPE table for P=%d D=%d", P, Dp);
    }
    const int R = Bi > Bt ? Bi : Bt;
    CE_TRY(grow_buffer(h->pool, h->pool_bytes, ce::pacl_pool_part_bytes(R, P, Dp)));
    return timed(h, s, "pacl_pool", 2.0 * R * P * Dp * (weight_mode ? 2 : 1),
                 (double)Bi * P * Dp * (vp_dtype == CE_BF16 ? 2 : 4) + 4.0 * Bt * Dp + 4.0 * R * Dp,
                 [&] { return ce::launch_pacl_pool(visual_proj, vp_dtype == CE_BF16, Bi, P, text_proj, Bt, Dp,
                                                   weight_mode, rc, rs, out_img, out_txt, (float*)h->pool, s); });
}

int ce_pacl_forward(ce_handle* h, void* stream, const void* pixels, int pixel_dtype, int Bi, const int64_t* ids,
                    int Bt, int weight_mode, int rope, float* out_img, float* out_txt) {
    if (!h || !pixels || !ids || !out_img) return fail(CE_ERR_INVALID, "ce_pacl_forward: null argument");
    if (h->cfg.pacl_dim <= 0) return fail(CE_ERR_STATE, "ce_pacl_forward: handle has no PACL head");
    if (Bi <= 0 || Bt <= 0) return fail(CE_ERR_INVALID, "ce_pacl_forward: bad sizes");
    if (!(Bi == Bt || Bi == 1 || Bt == 1))
        return fail(CE_ERR_INVALID, "ce_pacl_forward: cannot broadcast %d images against %d texts", Bi, Bt);
    if (pixel_dtype != CE_F32 && pixel_dtype != CE_BF16) return fail(CE_ERR_INVALID, "ce_pacl_forward: pixel dtype");
    if (rope != CE_ROPE_NONE && rope != CE_ROPE_BEFORE && rope != CE_ROPE_AFTER)
        return fail(CE_ERR_INVALID, "ce_pacl_forward: unknown rope mode %d", rope);
    if (rope == CE_ROPE_AFTER && weight_mode != CE_PACL_SIGMOID10)
        return fail(CE_ERR_INVALID, "ce_pacl_forward: rope AFTER only affects the sigmoid10 activations");
    CE_TRY(check_ready(h, true));
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    const ce_config& c = h->cfg;
    const int E = c.embed_dim, Pd = c.pacl_dim, Dv = c.vision.width;
    const long P = (long)h->G * h->G, Lv = P + 1;
    // aux (must survive both towers): tclip [Bt,E] | tp [Bt,Pd]
    CE_TRY(ensure_ws(h, std::max(vision_bytes(h, Bi), text_bytes(h, Bt))));
    CE_TRY(ensure_tmp(h, align256((size_t)Bt * E * 4) + align256((size_t)Bt * Pd * 4) + align256((size_t)Bt * E * 4)));
    float* tclip = (float*)h->tmp;
    float* tp = (float*)(h->tmp + align256((size_t)Bt * E * 4));
    // 1) text tower + PACL text head (pacl.py:116-118)
    {
        TowerWs w = carve(h->ws, (long)Bt * c.context_length, c.text.width, c.text.mlp_width, 0, Bt);
        CE_TRY(run_text(h, s, w, ids, Bt, tclip, false, false));
        float* ln = (float*)h->tmp + 0;
        ln = (float*)(h->tmp + align256((size_t)Bt * E * 4) + align256((size_t)Bt * Pd * 4));
        CE_TRY(check_launch(ce::launch_ln_gather(ln, tclip, nullptr, E, Bt, E, W(h, "text_projection.0.weight"),
                                                 W(h, "text_projection.0.bias"), s), "pacl text ln"));
        ce::FGemmParams fp{};
        fp.A = ln; fp.lda = E; fp.B = W(h, "text_projection.2.weight"); fp.ldb = Pd; fp.C = tp; fp.ldc = Pd;
        fp.M = Bt; fp.N = Pd; fp.K = E; fp.batch = 1; fp.alpha = 1.f; fp.bias = W(h, "text_projection.2.bias");
        CE_TRY(check_launch(ce::launch_fgemm(fp, false, s), "pacl text linear"));
    }
    // 2) vision tower, tokens -> ln_post -> [rope] -> PACL LN (one fused row kernel) -> heads
    TowerWs w = carve(h->ws, Bi * Lv, Dv, c.vision.mlp_width, Bi * P * h->Kp, Bi);
    CE_TRY(run_vision(h, s, w, pixels, pixel_dtype == CE_BF16, Bi, nullptr, false));
    const int M = (int)(Bi * P);
    CE_TRY(layernorm(h, s, "ln_pacl", w.x, w.xn, true, W(h, "visual.ln_post.weight"), W(h, "visual.ln_post.bias"), M,
                     Dv, (int)P, (int)Lv, 1, (int)P, 0, W(h, "visual_projection.0.weight"),
                     W(h, "visual_projection.0.bias"), rope == CE_ROPE_BEFORE ? h->rc_v : nullptr,
                     rope == CE_ROPE_BEFORE ? h->rs_v : nullptr, (int)P));
    float* lin = (float*)w.qkv;          // [M, Pd] f32   (fits: Lv*3*Dv*2 >= P*Pd*4)
    bf16_t* h1 = w.att;                  // [M, Pd] bf16
    bf16_t* vp = w.hid;                  // [M, Pd] bf16
    CE_TRY(gemm(h, s, "gemm_pacl", w.xn, Dv, W<bf16_t>(h, "visual_projection.2.linear_projection.0.weight"), M, Pd, Dv,
                W(h, "visual_projection.2.linear_projection.0.bias"), ce::ACT_NONE_, nullptr, lin, false));
    CE_TRY(gemm(h, s, "gemm_pacl", w.xn, Dv, W<bf16_t>(h, "visual_projection.2.non_linear_projection.0.weight"), M, Pd,
                Dv, W(h, "visual_projection.2.non_linear_projection.0.bias"), ce::ACT_GELU_, nullptr, h1, true));
    CE_TRY(gemm(h, s, "gemm_pacl", h1, Pd, W<bf16_t>(h, "visual_projection.2.non_linear_projection.2.weight"), M, Pd,
                Pd, W(h, "visual_projection.2.non_linear_projection.2.bias"), ce::ACT_NONE_, lin, vp, true));
    // 3) fused patch alignment + pooling + normalise
    return ce_pacl_pool(h, stream, vp, CE_BF16, Bi, (int)P, tp, Bt, Pd, weight_mode, rope == CE_ROPE_AFTER, out_img,
                        out_txt);
}

int ce_sparc_forward(ce_handle* h, void* stream, const float* v, const float* l, int B, int P, int T, int D,
                     float sigma, float* out_grouped, float* out_l_norm, float* out_sim) {
    if (!h || !v || !l || !out_grouped) return fail(CE_ERR_INVALID, "ce_sparc_forward: null argument");
    if (B <= 0 || P <= 0 || T <= 0 || D <= 0) return fail(CE_ERR_INVALID, "ce_sparc_forward: bad sizes");
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    CE_TRY(ensure_tmp(h, (size_t)B * T * P * 4));
    float* sim = (float*)h->tmp;
    ce::FGemmParams a{};
    a.A = l; a.lda = D; a.sA = (long)T * D;
    a.B = v; a.ldb = D; a.sB = (long)P * D;
    a.C = sim; a.ldc = P; a.sC = (long)T * P;
    a.M = T; a.N = P; a.K = D; a.batch = B; a.alpha = 1.f;
    CE_TRY(timed(h, s, "sparc_sim", 2.0 * B * T * P * D, 4.0 * B * ((double)T * D + (double)P * D + (double)T * P),
                 [&] { return ce::launch_fgemm(a, true, s); }));
    if (out_sim) HIP_TRY(hipMemcpyAsync(out_sim, sim, (size_t)B * T * P * 4, hipMemcpyDeviceToDevice, s));
    CE_TRY(check_launch(ce::launch_sparc_weights(sim, (long)B * T, P, sigma, s), "sparc weights"));
    ce::FGemmParams b{};
    b.A = sim; b.lda = P; b.sA = (long)T * P;
    b.B = v; b.ldb = D; b.sB = (long)P * D;
    b.C = out_grouped; b.ldc = D; b.sC = (long)T * D;
    b.M = T; b.N = D; b.K = P; b.batch = B; b.alpha = 1.f;
    CE_TRY(timed(h, s, "sparc_group", 2.0 * B * T * P * D, 4.0 * B * ((double)T * P + (double)P * D + (double)T * D),
                 [&] { return ce::launch_fgemm(b, false, s); }));
    CE_TRY(check_launch(ce::launch_l2norm(out_grouped, out_grouped, B * T, D, s), "normalize"));
    if (out_l_norm) CE_TRY(check_launch(ce::launch_l2norm(out_l_norm, l, B * T, D, s), "normalize"));
    return CE_OK;
}

namespace {

// Rows [row0, row0 + B) of the global CLIP loss of ClipLoss.forward (pacl.py:498-512) both ways:
// Li = scale img_all[row0..] txt_all^T, Lt = scale txt_all[row0..] img_all^T ([B, Bg] each), per-row CE
// against labels arange + row0 into lr / lc.  One shard (B == Bg): one fused launch for both ways.
int contrastive_rows(ce_handle* h, hipStream_t s, const float* img_all, const float* txt_all, int Bg, int row0, int B,
                     int D, float scale, float* Li, float* Lt, float* lr, float* lc) {
    ce::FGemmParams a{};
    a.A = img_all + (size_t)row0 * D; a.lda = D; a.B = txt_all; a.ldb = D; a.C = Li; a.ldc = Bg;
    a.M = B; a.N = Bg; a.K = D; a.batch = 1; a.alpha = scale;
    if (B == Bg) { a.Ct = Lt; a.ldct = Bg; }
    CE_TRY(check_launch(ce::launch_fgemm(a, true, s), "loss global logits"));
    if (B != Bg) {
        ce::FGemmParams b = a;
        b.A = txt_all + (size_t)row0 * D; b.B = img_all; b.C = Lt;
        CE_TRY(check_launch(ce::launch_fgemm(b, true, s), "loss global logits"));
    }
    CE_TRY(check_launch(ce::launch_ce_diag_rows(lr, Li, B, Bg, row0, s), "loss ce"));
    return check_launch(ce::launch_ce_diag_rows(lc, Lt, B, Bg, row0, s), "loss ce");
}

// SparcLoss's masked pairwise local loss of B samples (pacl.py:522-556,575-580): S[b] = scale grouped[b]
// l[b]^T, per-sample masked row / column CE sums into part[B][3]
int sparc_local_part(ce_handle* h, hipStream_t s, const float* l_tokens, const float* grouped, const float* mask, int B,
                     int T, int D, float scale, float* S, float* part) {
    ce::FGemmParams c{};
    c.A = grouped; c.lda = D; c.sA = (long)T * D;
    c.B = l_tokens; c.ldb = D; c.sB = (long)T * D;
    c.C = S; c.ldc = T; c.sC = (long)T * T;
    c.M = T; c.N = T; c.K = D; c.batch = B; c.alpha = scale;
    CE_TRY(timed(h, s, "sparc_loss_local", 2.0 * B * T * T * D, 4.0 * B * (2.0 * T * D + (double)T * T),
                 [&] { return ce::launch_fgemm(c, true, s); }));
    return check_launch(ce::launch_sparc_local(part, S, mask, B, T, s), "sparc_loss local");
}

int sparc_means(hipStream_t s, const float* v_patch, const float* l_tokens, int B, int P, int T, int D, float* gi,
                float* gt) {
    CE_TRY(check_launch(ce::launch_mean_mid(gi, v_patch, B, P, D, s), "sparc_loss mean"));
    CE_TRY(check_launch(ce::launch_mean_mid(gt, l_tokens, B, T, D, s), "sparc_loss mean"));
    CE_TRY(check_launch(ce::launch_l2norm(gi, gi, B, D, s), "sparc_loss normalize"));
    return check_launch(ce::launch_l2norm(gt, gt, B, D, s), "sparc_loss normalize");
}

int check_shard(const char* fn, int Bg, int row0, int B, int D) {
    if (B <= 0 || D <= 0 || Bg <= 0 || row0 < 0 || row0 + B > Bg)
        return fail(CE_ERR_INVALID, "%s: shard rows [%d, %d) outside the global batch of %d (D %d)", fn, row0,
                    row0 + B, Bg, D);
    return CE_OK;
}

}  // namespace

int ce_sparc_loss(ce_handle* h, void* stream, const float* v_patch, const float* l_tokens, const float* grouped,
                  const float* mask, int B, int P, int T, int D, float temperature, float global_weight,
                  float local_weight, float* out_loss) {
    if (!h || !v_patch || !l_tokens || !grouped || !mask || !out_loss)
        return fail(CE_ERR_INVALID, "ce_sparc_loss: null argument");
    if (B <= 0 || P <= 0 || T <= 0 || D <= 0 || !(temperature > 0.f))
        return fail(CE_ERR_INVALID, "ce_sparc_loss: bad sizes or temperature");
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    const float scale = 1.0f / temperature;   // ClipLoss.logit_scale (pacl.py:491-493)
    const size_t nGI = (size_t)B * D, nG = (size_t)B * B, nS = (size_t)B * T * T;
    CE_TRY(ensure_tmp(h, (2 * nGI + 2 * nG + nS + 5 * (size_t)B + 8) * 4));
    float* gi = (float*)h->tmp;
    float* gt = gi + nGI;
    float* G = gt + nGI;
    float* Gt = G + nG;
    float* S = Gt + nG;
    float* lr = S + nS;
    float* lc = lr + B;
    float* part = lc + B;
    float* parts = part + 3 * (size_t)B;
    // the whole batch is one shard: global term over the B x B logits, local term, combine
    CE_TRY(sparc_means(s, v_patch, l_tokens, B, P, T, D, gi, gt));
    CE_TRY(contrastive_rows(h, s, gi, gt, B, 0, B, D, scale, G, Gt, lr, lc));
    CE_TRY(sparc_local_part(h, s, l_tokens, grouped, mask, B, T, D, scale, S, part));
    CE_TRY(check_launch(ce::launch_loss_parts(parts, lr, lc, B, part, B, s), "sparc_loss parts"));
    return check_launch(ce::launch_loss_combine(out_loss, parts, B, global_weight, local_weight, s),
                        "sparc_loss combine");
}

int ce_sparc_loss_means(ce_handle* h, void* stream, const float* v_patch, const float* l_tokens, int B, int P, int T,
                        int D, float* out_img, float* out_txt) {
    if (!h || !v_patch || !l_tokens || !out_img || !out_txt) return fail(CE_ERR_INVALID, "ce_sparc_loss_means: null argument");
    if (B <= 0 || P <= 0 || T <= 0 || D <= 0) return fail(CE_ERR_INVALID, "ce_sparc_loss_means: bad sizes");
    DeviceGuard g(h->device);
    return sparc_means((hipStream_t)stream, v_patch, l_tokens, B, P, T, D, out_img, out_txt);
}

int ce_sparc_loss_partial(ce_handle* h, void* stream, const float* img_all, const float* txt_all, int Bg, int row0,
                          const float* l_tokens, const float* grouped, const float* mask, int B, int T, int D,
                          float temperature, float* parts) {
    if (!h || !img_all || !txt_all || !l_tokens || !grouped || !mask || !parts)
        return fail(CE_ERR_INVALID, "ce_sparc_loss_partial: null argument");
    if (T <= 0 || !(temperature > 0.f)) return fail(CE_ERR_INVALID, "ce_sparc_loss_partial: bad sizes or temperature");
    CE_TRY(check_shard("ce_sparc_loss_partial", Bg, row0, B, D));
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    const float scale = 1.0f / temperature;
    const size_t nL = (size_t)B * Bg, nS = (size_t)B * T * T;
    CE_TRY(ensure_tmp(h, (2 * nL + nS + 5 * (size_t)B) * 4));
    float* Li = (float*)h->tmp;
    float* Lt = Li + nL;
    float* S = Lt + nL;
    float* lr = S + nS;
    float* lc = lr + B;
    float* part = lc + B;
    CE_TRY(contrastive_rows(h, s, img_all, txt_all, Bg, row0, B, D, scale, Li, Lt, lr, lc));
    CE_TRY(sparc_local_part(h, s, l_tokens, grouped, mask, B, T, D, scale, S, part));
    return check_launch(ce::launch_loss_parts(parts, lr, lc, B, part, B, s), "sparc_loss parts");
}

int ce_contrastive_loss_partial(ce_handle* h, void* stream, const float* img_all, const float* txt_all, int Bg,
                                int row0, int B, int D, float scale, float* parts) {
    if (!h || !img_all || !txt_all || !parts) return fail(CE_ERR_INVALID, "ce_contrastive_loss_partial: null argument");
    CE_TRY(check_shard("ce_contrastive_loss_partial", Bg, row0, B, D));
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    const size_t nL = (size_t)B * Bg;
    CE_TRY(ensure_tmp(h, (2 * nL + 2 * (size_t)B) * 4));
    float* Li = (float*)h->tmp;
    float* Lt = Li + nL;
    float* lr = Lt + nL;
    float* lc = lr + B;
    CE_TRY(contrastive_rows(h, s, img_all, txt_all, Bg, row0, B, D, scale, Li, Lt, lr, lc));
    return check_launch(ce::launch_loss_parts(parts, lr, lc, B, nullptr, 0, s), "contrastive parts");
}

int ce_loss_combine(ce_handle* h, void* stream, const float* parts, int n_global, float global_weight,
                    float local_weight, float* out_loss) {
    if (!h || !parts || !out_loss) return fail(CE_ERR_INVALID, "ce_loss_combine: null argument");
    if (n_global <= 0) return fail(CE_ERR_INVALID, "ce_loss_combine: bad global batch %d", n_global);
    DeviceGuard g(h->device);
    return check_launch(ce::launch_loss_combine(out_loss, parts, n_global, global_weight, local_weight,
                                                (hipStream_t)stream), "loss combine");
}

// ---------------------------------------------------------------------------------------------
// Device preprocessing (preprocess.hip).  Tap tables are built here exactly as the reference's
// third-party resamplers build them: Pillow's precompute_coeffs + normalize_coeffs_8bpc (double
// precision, 22-bit fixed point) for the CLIP bicubic path, ATen's _compute_weights_aa (float,
// with its double-precision intermediates) for the PACL antialiased-bilinear path.
namespace {

double pil_bicubic(double x) {
    const double a = -0.5;
    if (x < 0.0) x = -x;
    if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
    if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
    return 0.0;
}

// Taps of output indices [o0, o0 + n) of an in_size -> out_size resize; bounds are (start, count)
// with start shifted by -shift.  Returns the tap row stride.
int pil_taps(int in_size, int out_size, int o0, int n, int shift, std::vector<int>& bounds, std::vector<int>& taps) {
    if (in_size == out_size) {            // Pillow skips the pass: identity taps reproduce it exactly
        for (int i = 0; i < n; ++i) {
            bounds.push_back(o0 + i - shift);
            bounds.push_back(1);
            taps.push_back(1 << 22);
        }
        return 1;
    }
    const double scale = (double)((float)in_size - 0.0f) / out_size;
    const double filterscale = scale < 1.0 ? 1.0 : scale;
    const double support = 2.0 * filterscale;
    const int ksize = (int)std::ceil(support) * 2 + 1;
    std::vector<double> k(ksize);
    for (int i = 0; i < n; ++i) {
        const int xx = o0 + i;
        const double center = 0.0 + (xx + 0.5) * scale;
        const double ss = 1.0 / filterscale;
        int xmin = (int)(center - support + 0.5);
        if (xmin < 0) xmin = 0;
        int xmax = (int)(center + support + 0.5);
        if (xmax > in_size) xmax = in_size;
        xmax -= xmin;
        double ww = 0.0;
        for (int x = 0; x < xmax; ++x) {
            k[x] = pil_bicubic((x + xmin - center + 0.5) * ss);
            ww += k[x];
        }
        for (int x = 0; x < ksize; ++x) {
            double v = x < xmax ? (ww != 0.0 ? k[x] / ww : k[x]) : 0.0;
            taps.push_back(v < 0 ? (int)(-0.5 + v * (1 << 22)) : (int)(0.5 + v * (1 << 22)));
        }
        bounds.push_back(xmin - shift);
        bounds.push_back(xmax);
    }
    return ksize;
}

int aa_taps(int in_size, int out_size, int shift, std::vector<int>& bounds, std::vector<float>& taps) {
    if (in_size == out_size) {            // ATen skips the dimension
        for (int i = 0; i < out_size; ++i) {
            bounds.push_back(i - shift);
            bounds.push_back(1);
            taps.push_back(1.0f);
        }
        return 1;
    }
    const float scale = (float)in_size / (float)out_size;
    const float support = scale >= 1.0f ? scale : 1.0f;
    const float invscale = scale >= 1.0f ? (float)(1.0 / (double)scale) : 1.0f;
    const int ksize = (int)std::ceil((double)support) * 2 + 1;
    std::vector<float> w(ksize);
    for (int i = 0; i < out_size; ++i) {
        const float center = (float)((double)scale * (i + 0.5));
        int xmin = (int)((double)(center - support) + 0.5);
        if (xmin < 0) xmin = 0;
        int xs = (int)((double)(center + support) + 0.5);
        if (xs > in_size) xs = in_size;
        xs -= xmin;
        float tot = 0.0f;
        for (int j = 0; j < xs; ++j) {
            float t = (float)(((double)((float)(j + xmin) - center) + 0.5) * (double)invscale);
            if (t < 0) t = -t;
            w[j] = t < 1.0f ? 1.0f - t : 0.0f;
            tot += w[j];
        }
        for (int j = 0; j < ksize; ++j) taps.push_back(j < xs ? (tot != 0.0f ? w[j] / tot : w[j]) : 0.0f);
        bounds.push_back(xmin - shift);
        bounds.push_back(xs);
    }
    return ksize;
}

int grow_pinned(char*& buf, size_t& bytes, size_t need) {
    if (need <= bytes) return CE_OK;
    if (buf) HIP_TRY(hipHostFree(buf));
    buf = nullptr;
    bytes = 0;
    if (hipHostMalloc((void**)&buf, need) != hipSuccess) {
        buf = nullptr;
        (void)hipGetLastError();
        return fail(CE_ERR_OOM, "cannot allocate %zu bytes of pinned staging", need);
    }
    bytes = need;
    return CE_OK;
}

}  // namespace

namespace {

// boxes: null, or per image (top, left, height, width) of a crop resized to S x S (CLIP bicubic only)
int preprocess_impl(ce_handle* h, void* stream, const uint8_t* images, const int64_t* offsets, const int* heights,
                    const int* widths, const int* boxes, int B, int mode, int out_dtype, void* out) {
    if (!h || !images || !offsets || !heights || !widths || !out)
        return fail(CE_ERR_INVALID, "ce_preprocess_images: null argument");
    if (B <= 0) return fail(CE_ERR_INVALID, "ce_preprocess_images: batch must be positive (got %d)", B);
    if (mode != CE_PRE_CLIP_BICUBIC && mode != CE_PRE_PACL_BILINEAR_AA)
        return fail(CE_ERR_INVALID, "ce_preprocess_images: unknown mode %d", mode);
    if (boxes && mode != CE_PRE_CLIP_BICUBIC)
        return fail(CE_ERR_INVALID, "ce_preprocess_images: crop boxes need the CLIP bicubic mode");
    if (out_dtype != CE_F32 && out_dtype != CE_BF16)
        return fail(CE_ERR_INVALID, "ce_preprocess_images: output must be f32 or bf16");
    const int S = h->cfg.image_size;
    const bool pacl = mode == CE_PRE_PACL_BILINEAR_AA;
    std::vector<ce::PrepMeta> meta(B);
    std::vector<int> bounds, itaps;
    std::vector<float> ftaps;
    long long tmp_elems = 0;
    int max_rows = 0;
    for (int b = 0; b < B; ++b) {
        const int H = heights[b], Wd = widths[b];
        if (H <= 0 || Wd <= 0 || offsets[b] < 0)
            return fail(CE_ERR_INVALID, "ce_preprocess_images: image %d has bad size %dx%d", b, H, Wd);
        ce::PrepMeta& m = meta[b];
        m.in_off = offsets[b];
        m.H = H;
        m.W = Wd;
        m.bx_off = (int)bounds.size();
        if (boxes) {
            // torchvision F.resized_crop on a PIL image: img.crop((left, top, left + w, top + h))
            // .resize((S, S), BICUBIC) -> Pillow's resampler over the crop, both axes to S
            const int top = boxes[4 * b], left = boxes[4 * b + 1], bh = boxes[4 * b + 2], bw = boxes[4 * b + 3];
            if (top < 0 || left < 0 || bh <= 0 || bw <= 0 || top + bh > H || left + bw > Wd)
                return fail(CE_ERR_INVALID, "ce_preprocess_images: crop box %d (%d,%d,%d,%d) outside the %dx%d image", b,
                            top, left, bh, bw, H, Wd);
            m.kx_off = (int)itaps.size();
            m.ksx = pil_taps(bw, S, 0, S, -left, bounds, itaps);
            std::vector<int> vb, vt;
            const int ksy = pil_taps(bh, S, 0, S, -top, vb, vt);
            m.ybase = vb[0];
            m.nrows = vb[2 * (S - 1)] + vb[2 * (S - 1) + 1] - m.ybase;
            for (int i = 0; i < S; ++i) vb[2 * i] -= m.ybase;
            m.by_off = (int)bounds.size();
            bounds.insert(bounds.end(), vb.begin(), vb.end());
            m.ky_off = (int)itaps.size();
            m.ksy = ksy;
            itaps.insert(itaps.end(), vt.begin(), vt.end());
        } else if (!pacl) {
            // torchvision Resize(S) shortest edge (_compute_resized_output_size) + CenterCrop(S)
            // offsets int(round(d / 2.0)) with round-half-even
            const bool wshort = Wd <= H;
            const int sh = wshort ? Wd : H, lg = wshort ? H : Wd;
            const int nl = (int)((double)S * lg / sh);
            const int nw = wshort ? S : nl, nh = wshort ? nl : S;
            const int top = (int)std::nearbyint((nh - S) / 2.0), left = (int)std::nearbyint((nw - S) / 2.0);
            m.kx_off = (int)itaps.size();
            m.ksx = pil_taps(Wd, nw, left, S, 0, bounds, itaps);
            // vertical taps first into scratch to learn the source row window
            std::vector<int> vb, vt;
            const int ksy = pil_taps(H, nh, top, S, 0, vb, vt);
            m.ybase = vb[0];
            m.nrows = vb[2 * (S - 1)] + vb[2 * (S - 1) + 1] - m.ybase;
            for (int i = 0; i < S; ++i) vb[2 * i] -= m.ybase;
            m.by_off = (int)bounds.size();
            bounds.insert(bounds.end(), vb.begin(), vb.end());
            m.ky_off = (int)itaps.size();
            m.ksy = ksy;
            itaps.insert(itaps.end(), vt.begin(), vt.end());
        } else {
            m.kx_off = (int)ftaps.size();
            m.ksx = aa_taps(Wd, S, 0, bounds, ftaps);
            std::vector<int> vb;
            std::vector<float> vt;
            const int ksy = aa_taps(H, S, 0, vb, vt);
            m.ybase = vb[0];
            m.nrows = vb[2 * (S - 1)] + vb[2 * (S - 1) + 1] - m.ybase;
            for (int i = 0; i < S; ++i) vb[2 * i] -= m.ybase;
            m.by_off = (int)bounds.size();
            bounds.insert(bounds.end(), vb.begin(), vb.end());
            m.ky_off = (int)ftaps.size();
            m.ksy = ksy;
            ftaps.insert(ftaps.end(), vt.begin(), vt.end());
        }
        m.tmp_off = tmp_elems;
        tmp_elems += (long long)m.nrows * S * 3;
        if (m.nrows > max_rows) max_rows = m.nrows;
    }
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    const size_t meta_b = (size_t)B * sizeof(ce::PrepMeta);
    const size_t bounds_b = bounds.size() * 4;
    const size_t taps_b = pacl ? ftaps.size() * 4 : itaps.size() * 4;
    const size_t total = meta_b + bounds_b + taps_b;
    if (h->prep_ev) HIP_TRY(hipEventSynchronize(h->prep_ev));     // staging buffer free again
    else HIP_TRY(hipEventCreateWithFlags(&h->prep_ev, hipEventDisableTiming));
    CE_TRY(grow_pinned(h->prep_host, h->prep_host_bytes, total));
    CE_TRY(grow_buffer(h->prep_dev, h->prep_dev_bytes, total));
    CE_TRY(grow_buffer(h->prep_tmp, h->prep_tmp_bytes, (size_t)tmp_elems * (pacl ? 4 : 1)));
    memcpy(h->prep_host, meta.data(), meta_b);
    memcpy(h->prep_host + meta_b, bounds.data(), bounds_b);
    memcpy(h->prep_host + meta_b + bounds_b, pacl ? (const void*)ftaps.data() : (const void*)itaps.data(), taps_b);
    HIP_TRY(hipMemcpyAsync(h->prep_dev, h->prep_host, total, hipMemcpyHostToDevice, s));
    HIP_TRY(hipEventRecord(h->prep_ev, s));
    static const float kOpenaiMean[3] = {0.48145466f, 0.4578275f, 0.40821073f};
    static const float kOpenaiStd[3] = {0.26862954f, 0.26130258f, 0.27577711f};
    static const float kImagenetMean[3] = {0.485f, 0.456f, 0.406f};
    static const float kImagenetStd[3] = {0.229f, 0.224f, 0.225f};
    return timed(h, s, "preprocess", 0.0, (double)tmp_elems * 2 + (double)B * 3 * S * S * (out_dtype == CE_BF16 ? 2 : 4),
                 [&] {
                     return ce::launch_preprocess(images, (const ce::PrepMeta*)h->prep_dev,
                                                  (const int*)(h->prep_dev + meta_b),
                                                  (const void*)(h->prep_dev + meta_b + bounds_b), h->prep_tmp, B,
                                                  max_rows, S, pacl, out_dtype == CE_BF16,
                                                  pacl ? kImagenetMean : kOpenaiMean, pacl ? kImagenetStd : kOpenaiStd,
                                                  out, s);
                 });
}

}  // namespace

int ce_preprocess_images(ce_handle* h, void* stream, const uint8_t* images, const int64_t* offsets,
                         const int* heights, const int* widths, int B, int mode, int out_dtype, void* out) {
    return preprocess_impl(h, stream, images, offsets, heights, widths, nullptr, B, mode, out_dtype, out);
}

int ce_preprocess_images_boxes(ce_handle* h, void* stream, const uint8_t* images, const int64_t* offsets,
                               const int* heights, const int* widths, const int* boxes, int B, int out_dtype,
                               void* out) {
    if (!boxes) return fail(CE_ERR_INVALID, "ce_preprocess_images_boxes: null boxes");
    return preprocess_impl(h, stream, images, offsets, heights, widths, boxes, B, CE_PRE_CLIP_BICUBIC, out_dtype, out);
}

// ---------------------------------------------------------------------------------------------
// SPARC head training (train_sparc.py:29-37,91,106; model/pacl.py:380-584).  Forward keeps the
// activations in h->sp; loss_grad takes the global loss's gradient w.r.t. this rank's normalised
// means and local-term inputs; backward runs it down to the 12 head tensors.
namespace {

const char* const kSparcHead[12] = {
    "visual_projection.0.weight", "visual_projection.0.bias",
    "visual_projection.2.linear_projection.0.weight", "visual_projection.2.linear_projection.0.bias",
    "visual_projection.2.non_linear_projection.0.weight", "visual_projection.2.non_linear_projection.0.bias",
    "visual_projection.2.non_linear_projection.2.weight", "visual_projection.2.non_linear_projection.2.bias",
    "text_projection.0.weight", "text_projection.0.bias", "text_projection.2.weight", "text_projection.2.bias"};

struct SparcWs {
    int B, P, T, Dv, E, Pd;
    long N1, Nt;
    float *xv, *ylin, *v, *xt, *ht, *l, *Ln, *S, *Wt, *G, *Gn, *mv, *ml, *dgi, *dgt, *R, *dR, *dRT, *part;
    float *dGn, *dLn, *dG, *dS, *tT, *dv, *dh, *dl, *dlT, *dht, *cs, *lng, *abw, *gpart, *dmv, *dml;
    float2 *stv, *stt;
    bf16_t *hv, *a, *g, *dvb, *da, *W2T, *WlT, *W1T;
};

size_t sparc_layout(const ce_handle* h, int B, int P, int T, SparcWs* w, char* base) {
    const ce_config& c = h->cfg;
    SparcWs t{};
    t.B = B; t.P = P; t.T = T; t.Dv = c.vision.width; t.E = c.embed_dim; t.Pd = c.pacl_dim;
    t.N1 = (long)B * P; t.Nt = (long)B * T;
    size_t off = 0;
    auto take = [&](size_t bytes) -> char* {
        char* r = base ? base + off : nullptr;
        off += align256(bytes);
        return r;
    };
    const long N1 = t.N1, Nt = t.Nt, Dv = t.Dv, E = t.E, Pd = t.Pd;
    const long BTP = (long)B * T * P, BTD = (long)B * T * Pd, BTT = (long)B * T * T;
    t.xv = (float*)take(N1 * Dv * 4);   t.stv = (float2*)take(N1 * 8);   t.hv = (bf16_t*)take(N1 * Dv * 2);
    t.a = (bf16_t*)take(N1 * Pd * 2);   t.g = (bf16_t*)take(N1 * Pd * 2);
    t.ylin = (float*)take(N1 * Pd * 4); t.v = (float*)take(N1 * Pd * 4);
    t.xt = (float*)take(Nt * E * 4);    t.stt = (float2*)take(Nt * 8);   t.ht = (float*)take(Nt * E * 4);
    t.l = (float*)take(Nt * Pd * 4);    t.Ln = (float*)take(Nt * Pd * 4);
    t.S = (float*)take(BTP * 4);        t.Wt = (float*)take(BTP * 4);
    t.G = (float*)take(BTD * 4);        t.Gn = (float*)take(BTD * 4);
    t.mv = (float*)take((long)B * Pd * 4); t.ml = (float*)take((long)B * Pd * 4);
    t.dgi = (float*)take((long)B * Pd * 4); t.dgt = (float*)take((long)B * Pd * 4);
    t.dmv = (float*)take((long)B * Pd * 4); t.dml = (float*)take((long)B * Pd * 4);
    t.R = (float*)take(BTT * 4);        t.dR = (float*)take(BTT * 4);    t.dRT = (float*)take(BTT * 4);
    t.part = (float*)take((long)B * 3 * 4 + 32);
    t.dGn = (float*)take(BTD * 4);      t.dLn = (float*)take(BTD * 4);   t.dG = (float*)take(BTD * 4);
    t.dS = (float*)take(BTP * 4);       t.tT = (float*)take(BTP * 4);
    t.dv = (float*)take(N1 * Pd * 4);   t.dvb = (bf16_t*)take(N1 * Pd * 2); t.da = (bf16_t*)take(N1 * Pd * 2);
    t.dh = (float*)take(N1 * Dv * 4);
    t.dl = (float*)take(Nt * Pd * 4);   t.dlT = (float*)take(Nt * Pd * 4); t.dht = (float*)take(Nt * E * 4);
    t.W2T = (bf16_t*)take(Pd * Pd * 2); t.WlT = (bf16_t*)take(Dv * Pd * 2); t.W1T = (bf16_t*)take(Dv * Pd * 2);
    t.cs = (float*)take(std::max(ce::colsum_scratch_floats((int)N1, (int)Pd), ce::colsum_scratch_floats((int)Nt, (int)Pd)) * 4);
    t.lng = (float*)take(std::max(ce::ln_grad_scratch_floats(N1, (int)Dv), ce::ln_grad_scratch_floats(Nt, (int)E)) * 4);
    t.abw = (float*)take(std::max(ce::act_bwd_colsum_scratch_floats((int)N1, (int)Pd), ((N1 + 127) / 128) * Pd) * 4);
    t.gpart = (float*)take(ce::kGemmPartElems * 4);
    if (w) *w = t;
    return off;
}

float* sp_param(ce_handle* h, const char* n) { return h->sp_bound.at(n).first; }
float* sp_grad(ce_handle* h, const char* n) { return h->sp_bound.at(n).second; }

int sparc_fgemm(ce_handle* h, hipStream_t s, const char* tag, const float* A, long lda, long sA, const float* B, long ldb,
                long sB, float* C, long ldc, long sC, int M, int N, int K, int batch, float alpha, bool b_nk,
                const float* bias = nullptr, bool accumulate = false) {
    ce::FGemmParams f{};
    f.A = A; f.lda = lda; f.sA = sA; f.B = B; f.ldb = ldb; f.sB = sB; f.C = C; f.ldc = ldc; f.sC = sC;
    f.M = M; f.N = N; f.K = K; f.batch = batch; f.alpha = alpha; f.bias = bias; f.accumulate = accumulate ? 1 : 0;
    return timed(h, s, tag, 2.0 * M * N * K * batch, 0.0, [&] { return ce::launch_fgemm(f, b_nk, s); });
}

}  // namespace

int ce_sparc_train_bind(ce_handle* h, const ce_tensor* params, const ce_tensor* grads, int n) {
    if (!h || (n > 0 && (!params || !grads))) return fail(CE_ERR_INVALID, "ce_sparc_train_bind: null argument");
    if (h->cfg.pacl_dim <= 0) return fail(CE_ERR_STATE, "ce_sparc_train_bind: handle has no PACL / SPARC head");
    std::map<std::string, std::pair<float*, float*>> b;
    for (int i = 0; i < n; ++i) {
        if (!params[i].name || !grads[i].name || strcmp(params[i].name, grads[i].name) != 0)
            return fail(CE_ERR_INVALID, "ce_sparc_train_bind: entry %d: params and grads must name the same tensor", i);
        const std::string name = canonical(h, params[i].name);
        if (std::find_if(std::begin(kSparcHead), std::end(kSparcHead), [&](const char* k) { return name == k; }) ==
            std::end(kSparcHead))
            return fail(CE_ERR_INVALID, "ce_sparc_train_bind: '%s' is not a SPARC head tensor", params[i].name);
        const WSpec& sp = h->specs.at(name);
        if (params[i].dtype != CE_F32 || grads[i].dtype != CE_F32 || !params[i].data || !grads[i].data)
            return fail(CE_ERR_INVALID, "ce_sparc_train_bind: '%s' needs f32 device buffers", params[i].name);
        for (const ce_tensor* t : {&params[i], &grads[i]}) {
            bool ok = t->ndim == (int)sp.shape.size();
            for (int d = 0; ok && d < t->ndim; ++d) ok = t->shape[d] == sp.shape[d];
            if (!ok) return fail(CE_ERR_INVALID, "ce_sparc_train_bind: '%s' has the wrong shape", params[i].name);
        }
        b[name] = {(float*)params[i].data, (float*)grads[i].data};
    }
    for (const char* k : kSparcHead)
        if (!b.count(k)) return fail(CE_ERR_INVALID, "ce_sparc_train_bind: head tensor '%s' not bound", k);
    h->sp_bound = b;
    h->sp_state = 0;
    return CE_OK;
}

int ce_sparc_train_sync_weights(ce_handle* h, void* stream) {
    if (!h) return fail(CE_ERR_INVALID, "ce_sparc_train_sync_weights: null handle");
    if (h->sp_bound.empty()) return fail(CE_ERR_STATE, "ce_sparc_train_sync_weights: no head bound (ce_sparc_train_bind)");
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    for (auto& kv : h->sp_bound) {
        const WSpec& sp = h->specs.at(kv.first);
        const size_t n = spec_elems(h, kv.first);
        void*& dp = h->dptr[kv.first];
        if (!dp) {
            if (hipMalloc(&dp, n * (sp.st == ST_BF16 ? 2 : 4)) != hipSuccess) {
                (void)hipGetLastError();
                h->dptr.erase(kv.first);
                return fail(CE_ERR_OOM, "ce_sparc_train_sync_weights: cannot allocate '%s'", kv.first.c_str());
            }
        }
        if (sp.st == ST_F32_T) {     // text_projection.2.weight [Pd][E] kept transposed for the f32 GEMM
            CE_TRY(check_launch(ce::launch_transpose_add(kv.second.first, nullptr, (float*)dp, 1, (int)sp.shape[0],
                                                         (int)sp.shape[1], s), "sparc weight sync"));
        } else if (sp.st == ST_BF16 || sp.st == ST_F32) {
            const long row = sp.shape.size() == 2 ? sp.shape[1] : 1;
            CE_TRY(check_launch(ce::launch_weight_from_master(dp, sp.st == ST_BF16, kv.second.first, (long)n, row, 0, 1.f, s),
                                "sparc weight sync"));
        } else {
            return fail(CE_ERR_INVALID, "ce_sparc_train_sync_weights: '%s' has an unsupported storage", kv.first.c_str());
        }
        h->loaded[kv.first] = true;
    }
    return CE_OK;
}

int ce_sparc_train_forward(ce_handle* h, void* stream, const float* patch_tokens, int B, int P, int rope,
                           const float* text, int text_mode, int T, float sigma, float dropout, uint64_t seed,
                           int64_t sample0, float* out_v, float* out_l, float* out_g) {
    if (!h || !patch_tokens || !text) return fail(CE_ERR_INVALID, "ce_sparc_train_forward: null argument");
    if (h->sp_bound.empty()) return fail(CE_ERR_STATE, "ce_sparc_train_forward: no head bound (ce_sparc_train_bind)");
    if (B <= 0 || P <= 0 || T <= 0 || T > 80) return fail(CE_ERR_INVALID, "ce_sparc_train_forward: bad sizes (T <= 80)");
    if (rope != CE_ROPE_NONE && rope != CE_ROPE_BEFORE) return fail(CE_ERR_INVALID, "ce_sparc_train_forward: rope NONE / BEFORE");
    if (rope == CE_ROPE_BEFORE && P != h->G * h->G)
        return fail(CE_ERR_INVALID, "ce_sparc_train_forward: rope tables cover %d patches", h->G * h->G);
    if (text_mode != 0 && text_mode != 1) return fail(CE_ERR_INVALID, "ce_sparc_train_forward: text_mode 0 or 1");
    if (!(dropout >= 0.f && dropout < 1.f)) return fail(CE_ERR_INVALID, "ce_sparc_train_forward: dropout in [0, 1)");
    if (sample0 < 0) return fail(CE_ERR_INVALID, "ce_sparc_train_forward: sample0 < 0");
    CE_TRY(check_ready(h, true));
    DeviceGuard dg(h->device);
    hipStream_t s = (hipStream_t)stream;
    CE_TRY(grow_buffer(h->sp, h->sp_bytes, sparc_layout(h, B, P, T, nullptr, nullptr)));
    SparcWs w;
    sparc_layout(h, B, P, T, &w, h->sp);
    const int Dv = w.Dv, E = w.E, Pd = w.Pd;
    const int N1 = (int)w.N1;
    h->sp_state = 0;
    // ---- visual head: [apply_rope] -> LayerNorm -> Dropout -> Patch_Projection (pacl.py:35-48,480-484) ----
    if (rope) CE_TRY(check_launch(ce::launch_rope(w.xv, patch_tokens, B, P, Dv, h->rc_v, h->rs_v, s), "sparc rope"));
    else HIP_TRY(hipMemcpyAsync(w.xv, patch_tokens, (size_t)w.N1 * Dv * 4, hipMemcpyDeviceToDevice, s));
    CE_TRY(timed(h, s, "sparc_ln_v", 0.0, 6.0 * w.N1 * Dv, [&] {
        return ce::launch_ln_drop(w.xv, W(h, "visual_projection.0.weight"), W(h, "visual_projection.0.bias"), w.N1, Dv,
                                  dropout, 2 * seed, (long)sample0 * P, w.hv, true, w.stv, s); }));
    CE_TRY(tgemm(h, s, "sparc_head_v", w.hv, Dv, W<bf16_t>(h, "visual_projection.2.linear_projection.0.weight"), Dv, N1,
                 Pd, Dv, W(h, "visual_projection.2.linear_projection.0.bias"), ce::ACT_NONE_, nullptr, w.ylin, false, w.gpart));
    {
        ce::GemmParams p{};     // GELU(Linear) with the pre-activation kept for the backward
        p.A = w.hv; p.lda = Dv; p.W = W<bf16_t>(h, "visual_projection.2.non_linear_projection.0.weight"); p.ldw = Dv;
        p.M = N1; p.N = Pd; p.K = Dv;
        p.bias = W(h, "visual_projection.2.non_linear_projection.0.bias");
        p.out = w.g; p.ldo = Pd; p.pre_out = w.a;
        p.part = w.gpart; p.part_elems = ce::kGemmPartElems;
        CE_TRY(timed(h, s, "sparc_head_v", 2.0 * N1 * Pd * Dv, 0.0, [&] { return ce::launch_gemm(p, ce::ACT_GELU_, true, s); }));
    }
    CE_TRY(tgemm(h, s, "sparc_head_v", w.g, Pd, W<bf16_t>(h, "visual_projection.2.non_linear_projection.2.weight"), Pd, N1,
                 Pd, Pd, W(h, "visual_projection.2.non_linear_projection.2.bias"), ce::ACT_NONE_, w.ylin, w.v, false, w.gpart));
    // ---- text: text_projection = LayerNorm -> Dropout -> Linear (pacl.py:431-436), or the embeddings ----
    if (text_mode == 0) {
        HIP_TRY(hipMemcpyAsync(w.xt, text, (size_t)w.Nt * E * 4, hipMemcpyDeviceToDevice, s));
        CE_TRY(timed(h, s, "sparc_ln_t", 0.0, 8.0 * w.Nt * E, [&] {
            return ce::launch_ln_drop(w.xt, W(h, "text_projection.0.weight"), W(h, "text_projection.0.bias"), w.Nt, E,
                                      dropout, 2 * seed + 1, (long)sample0 * T, w.ht, false, w.stt, s); }));
        CE_TRY(sparc_fgemm(h, s, "sparc_head_t", w.ht, E, 0, sp_param(h, "text_projection.2.weight"), E, 0, w.l, Pd, 0,
                           (int)w.Nt, Pd, E, 1, 1.f, true, W(h, "text_projection.2.bias")));
    } else {
        HIP_TRY(hipMemcpyAsync(w.l, text, (size_t)w.Nt * Pd * 4, hipMemcpyDeviceToDevice, s));
    }
    CE_TRY(check_launch(ce::launch_l2norm(w.Ln, w.l, (int)w.Nt, Pd, s), "sparc normalize"));
    // ---- alignment (pacl.py:455-476) ----
    CE_TRY(sparc_fgemm(h, s, "sparc_sim", w.l, Pd, (long)T * Pd, w.v, Pd, (long)P * Pd, w.S, P, (long)T * P, T, P, Pd, B,
                       1.f, true));
    HIP_TRY(hipMemcpyAsync(w.Wt, w.S, (size_t)B * T * P * 4, hipMemcpyDeviceToDevice, s));
    CE_TRY(check_launch(ce::launch_sparc_weights(w.Wt, (long)B * T, P, sigma, s), "sparc weights"));
    CE_TRY(sparc_fgemm(h, s, "sparc_group", w.Wt, P, (long)T * P, w.v, Pd, (long)P * Pd, w.G, Pd, (long)T * Pd, T, Pd, P,
                       B, 1.f, false));
    CE_TRY(check_launch(ce::launch_l2norm(w.Gn, w.G, B * T, Pd, s), "sparc normalize"));
    if (out_v) HIP_TRY(hipMemcpyAsync(out_v, w.v, (size_t)w.N1 * Pd * 4, hipMemcpyDeviceToDevice, s));
    if (out_l) HIP_TRY(hipMemcpyAsync(out_l, w.Ln, (size_t)w.Nt * Pd * 4, hipMemcpyDeviceToDevice, s));
    if (out_g) HIP_TRY(hipMemcpyAsync(out_g, w.Gn, (size_t)B * T * Pd * 4, hipMemcpyDeviceToDevice, s));
    h->sp_B = B; h->sp_P = P; h->sp_T = T; h->sp_text = text_mode;
    h->sp_sigma = sigma; h->sp_drop = dropout; h->sp_seed = seed; h->sp_sample0 = sample0;
    h->sp_state = 1;
    return CE_OK;
}

int ce_sparc_train_loss_grad(ce_handle* h, void* stream, const float* img_all, const float* txt_all, int Bg, int row0,
                             const float* mask, float mask_total, float temperature, float global_weight,
                             float local_weight, float* parts) {
    if (!h || !img_all || !txt_all || !mask || !parts) return fail(CE_ERR_INVALID, "ce_sparc_train_loss_grad: null argument");
    if (h->sp_state < 1) return fail(CE_ERR_STATE, "ce_sparc_train_loss_grad: no ce_sparc_train_forward before it");
    const int B = h->sp_B, T = h->sp_T;
    CE_TRY(check_shard("ce_sparc_train_loss_grad", Bg, row0, B, h->cfg.pacl_dim));
    if (!(temperature > 0.f) || !(mask_total > 0.f)) return fail(CE_ERR_INVALID, "ce_sparc_train_loss_grad: temperature / mask_total");
    DeviceGuard dg(h->device);
    hipStream_t s = (hipStream_t)stream;
    SparcWs w;
    sparc_layout(h, B, h->sp_P, T, &w, h->sp);
    const int Pd = w.Pd;
    const float scale = 1.0f / temperature;
    // local term (pacl.py:522-556,575-580): R = scale Gn Ln^T, dR, dGn = scale dR Ln, dLn = scale dR^T Gn
    CE_TRY(sparc_fgemm(h, s, "sparc_loss_local", w.Gn, Pd, (long)T * Pd, w.Ln, Pd, (long)T * Pd, w.R, T, (long)T * T, T, T,
                       Pd, B, scale, true));
    CE_TRY(check_launch(ce::launch_local_grad(w.R, mask, B, T, local_weight * 0.5f / mask_total, w.dR, w.dRT, w.part, s),
                        "sparc local grad"));
    CE_TRY(sparc_fgemm(h, s, "sparc_loss_local", w.dR, T, (long)T * T, w.Ln, Pd, (long)T * Pd, w.dGn, Pd, (long)T * Pd, T, Pd,
                       T, B, scale, false));
    CE_TRY(sparc_fgemm(h, s, "sparc_loss_local", w.dRT, T, (long)T * T, w.Gn, Pd, (long)T * Pd, w.dLn, Pd, (long)T * Pd, T,
                       Pd, T, B, scale, false));
    // global term (pacl.py:563-570) over the whole gathered batch (every rank computes the Bg x Bg
    // softmaxes; its rows of the gradient are this rank's): M = dLi + dLt^T
    const size_t nL = (size_t)Bg * Bg;
    CE_TRY(ensure_tmp(h, (6 * nL + 2 * (size_t)Bg) * 4));
    float* Li = (float*)h->tmp;
    float* Lt = Li + nL;
    float* dLi = Lt + nL;
    float* dLt = dLi + nL;
    float* M = dLt + nL;
    float* MT = M + nL;
    float* lr = MT + nL;
    float* lc = lr + Bg;
    {
        ce::FGemmParams a{};
        a.A = img_all; a.lda = Pd; a.B = txt_all; a.ldb = Pd; a.C = Li; a.ldc = Bg; a.Ct = Lt; a.ldct = Bg;
        a.M = Bg; a.N = Bg; a.K = Pd; a.batch = 1; a.alpha = scale;
        CE_TRY(check_launch(ce::launch_fgemm(a, true, s), "sparc global logits"));
    }
    const float wg = global_weight * 0.5f / (float)Bg;
    CE_TRY(check_launch(ce::launch_ce_diag_grad(Li, Bg, Bg, wg, dLi, lr, s), "sparc global grad"));
    CE_TRY(check_launch(ce::launch_ce_diag_grad(Lt, Bg, Bg, wg, dLt, lc, s), "sparc global grad"));
    CE_TRY(check_launch(ce::launch_transpose_add(dLt, dLi, M, 1, Bg, Bg, s), "sparc global grad"));
    CE_TRY(check_launch(ce::launch_transpose_add(dLi, dLt, MT, 1, Bg, Bg, s), "sparc global grad"));
    CE_TRY(sparc_fgemm(h, s, "sparc_loss_global", M + (size_t)row0 * Bg, Bg, 0, txt_all, Pd, 0, w.dgi, Pd, 0, B, Pd, Bg, 1,
                       scale, false));
    CE_TRY(sparc_fgemm(h, s, "sparc_loss_global", MT + (size_t)row0 * Bg, Bg, 0, img_all, Pd, 0, w.dgt, Pd, 0, B, Pd, Bg, 1,
                       scale, false));
    CE_TRY(check_launch(ce::launch_loss_parts(parts, lr + row0, lc + row0, B, w.part, B, s), "sparc loss parts"));
    h->sp_state = 2;
    return CE_OK;
}

int ce_sparc_train_backward(ce_handle* h, void* stream) {
    if (!h) return fail(CE_ERR_INVALID, "ce_sparc_train_backward: null handle");
    if (h->sp_state < 2) return fail(CE_ERR_STATE, "ce_sparc_train_backward: needs ce_sparc_train_forward + _loss_grad first");
    DeviceGuard dg(h->device);
    hipStream_t s = (hipStream_t)stream;
    const int B = h->sp_B, P = h->sp_P, T = h->sp_T;
    SparcWs w;
    sparc_layout(h, B, P, T, &w, h->sp);
    const int Dv = w.Dv, E = w.E, Pd = w.Pd, N1 = (int)w.N1, Nt = (int)w.Nt;
    const float p = h->sp_drop;
    const uint64_t seed = h->sp_seed;
    // ---- means + normalise (pacl.py:566-567) ----
    CE_TRY(check_launch(ce::launch_mean_mid(w.mv, w.v, B, P, Pd, s), "sparc bwd"));
    CE_TRY(check_launch(ce::launch_mean_mid(w.ml, w.Ln, B, T, Pd, s), "sparc bwd"));
    // (their own buffers: dR / dRT hold B x T x T floats, fewer than B x Pd for T < 28 -- one token per
    // caption in the PACL step)
    float* dmv = w.dmv;
    float* dml = w.dml;
    CE_TRY(check_launch(ce::launch_l2norm_bwd(dmv, w.mv, w.dgi, B, Pd, s), "sparc bwd"));
    CE_TRY(check_launch(ce::launch_l2norm_bwd(dml, w.ml, w.dgt, B, Pd, s), "sparc bwd"));
    CE_TRY(check_launch(ce::launch_bcast_add_mid(w.dLn, dml, B, T, Pd, 1.0f / T, s), "sparc bwd"));
    // ---- alignment (pacl.py:455-476) ----
    CE_TRY(check_launch(ce::launch_l2norm_bwd(w.dG, w.G, w.dGn, B * T, Pd, s), "sparc bwd"));
    // dW = dG v^T; dv = W^T dG
    CE_TRY(sparc_fgemm(h, s, "sparc_bwd_align", w.dG, Pd, (long)T * Pd, w.v, Pd, (long)P * Pd, w.dS, P, (long)T * P, T, P,
                       Pd, B, 1.f, true));
    CE_TRY(check_launch(ce::launch_transpose_add(w.Wt, nullptr, w.tT, B, T, P, s), "sparc bwd"));
    CE_TRY(sparc_fgemm(h, s, "sparc_bwd_align", w.tT, T, (long)P * T, w.dG, Pd, (long)T * Pd, w.dv, Pd, (long)P * Pd, P, Pd,
                       T, B, 1.f, false));
    CE_TRY(check_launch(ce::launch_align_bwd(w.S, w.dS, (long)B * T, P, h->sp_sigma, s), "sparc align bwd"));
    // dl = dS v; dv += dS^T l; dv += d mean_v / P
    CE_TRY(sparc_fgemm(h, s, "sparc_bwd_align", w.dS, P, (long)T * P, w.v, Pd, (long)P * Pd, w.dl, Pd, (long)T * Pd, T, Pd,
                       P, B, 1.f, false));
    CE_TRY(check_launch(ce::launch_transpose_add(w.dS, nullptr, w.tT, B, T, P, s), "sparc bwd"));
    CE_TRY(sparc_fgemm(h, s, "sparc_bwd_align", w.tT, T, (long)P * T, w.l, Pd, (long)T * Pd, w.dv, Pd, (long)P * Pd, P, Pd,
                       T, B, 1.f, false, nullptr, true));
    CE_TRY(check_launch(ce::launch_bcast_add_mid(w.dv, dmv, B, P, Pd, 1.0f / P, s), "sparc bwd"));
    // dl += normalize backward of dLn
    CE_TRY(check_launch(ce::launch_l2norm_bwd(w.dG, w.l, w.dLn, Nt, Pd, s), "sparc bwd"));
    CE_TRY(check_launch(ce::launch_axpy(w.dl, w.dG, (long)Nt * Pd, 1.f, s), "sparc bwd"));
    // ---- text head: Linear, Dropout, LayerNorm (f32) ----
    if (h->sp_text == 0) {
        CE_TRY(check_launch(ce::launch_colsum(sp_grad(h, "text_projection.2.bias"), w.dl, true, Pd, Nt, Pd, 1.f, false, w.cs, s),
                            "sparc bwd"));
        CE_TRY(check_launch(ce::launch_transpose_add(w.dl, nullptr, w.dlT, 1, Nt, Pd, s), "sparc bwd"));
        CE_TRY(sparc_fgemm(h, s, "sparc_bwd_head_t", w.dlT, Nt, 0, w.ht, E, 0, sp_grad(h, "text_projection.2.weight"), E, 0,
                           Pd, E, Nt, 1, 1.f, false));
        CE_TRY(sparc_fgemm(h, s, "sparc_bwd_head_t", w.dl, Pd, 0, sp_param(h, "text_projection.2.weight"), E, 0, w.dht, E, 0,
                           Nt, E, Pd, 1, 1.f, false));
        CE_TRY(check_launch(ce::launch_ln_grad(w.dht, w.xt, w.stt, Nt, E, p, 2 * seed + 1, (long)h->sp_sample0 * T,
                                               sp_grad(h, "text_projection.0.weight"),
                                               sp_grad(h, "text_projection.0.bias"), w.lng, s), "sparc ln grad"));
    } else {
        for (const char* n : {"text_projection.0.weight", "text_projection.0.bias", "text_projection.2.weight",
                              "text_projection.2.bias"})
            HIP_TRY(hipMemsetAsync(sp_grad(h, n), 0, spec_elems(h, n) * 4, s));
    }
    // ---- visual head: Patch_Projection, Dropout, LayerNorm (bf16 GEMM operands, f32 accumulation) ----
    CE_TRY(check_launch(ce::launch_cast_bf16(w.dvb, w.dv, (long)N1 * Pd, s), "sparc bwd"));
    float* dbl = sp_grad(h, "visual_projection.2.linear_projection.0.bias");
    CE_TRY(check_launch(ce::launch_colsum(dbl, w.dv, true, Pd, N1, Pd, 1.f, false, w.cs, s), "sparc bwd"));
    HIP_TRY(hipMemcpyAsync(sp_grad(h, "visual_projection.2.non_linear_projection.2.bias"), dbl, (size_t)Pd * 4,
                           hipMemcpyDeviceToDevice, s));
    CE_TRY(tgemm_tn(h, s, "sparc_bwd_dw", w.dvb, Pd, w.g, Pd, Pd, Pd, N1,
                    sp_grad(h, "visual_projection.2.non_linear_projection.2.weight"), w.gpart));
    CE_TRY(tgemm_tn(h, s, "sparc_bwd_dw", w.dvb, Pd, w.hv, Dv, Pd, Dv, N1,
                    sp_grad(h, "visual_projection.2.linear_projection.0.weight"), w.gpart));
    CE_TRY(check_launch(ce::launch_transpose_bf16(w.W2T, Pd, W<bf16_t>(h, "visual_projection.2.non_linear_projection.2.weight"),
                                                  false, Pd, Pd, Pd, Pd, s), "sparc bwd"));
    CE_TRY(check_launch(ce::launch_transpose_bf16(w.WlT, Pd, W<bf16_t>(h, "visual_projection.2.linear_projection.0.weight"),
                                                  false, Dv, Pd, Dv, Pd, s), "sparc bwd"));
    CE_TRY(check_launch(ce::launch_transpose_bf16(w.W1T, Pd, W<bf16_t>(h, "visual_projection.2.non_linear_projection.0.weight"),
                                                  false, Dv, Pd, Dv, Pd, s), "sparc bwd"));
    // dA = GELU'(a) * (dv W2) and the GELU bias gradient, fused in the GEMM's epilogue where the four-wave
    // kernel takes the shape (as the text-tower backward's c_fc, capi.hip run_text_backward)
    float* db1 = sp_grad(h, "visual_projection.2.non_linear_projection.0.bias");
    {
        ce::GemmParams pb{};
        pb.A = w.dvb; pb.lda = Pd; pb.W = w.W2T; pb.ldw = Pd;
        pb.M = N1; pb.N = Pd; pb.K = Pd;
        pb.out = w.da; pb.ldo = Pd;
        pb.bwd_pre = w.a; pb.bwd_part = w.abw;
        if (ce::gemm_act_bwd_fused(pb, ce::ACT_GELU_)) {
            CE_TRY(timed(h, s, "sparc_bwd_dx", 2.0 * N1 * Pd * Pd, 0.0, [&] { return ce::launch_gemm_act_bwd(pb, ce::ACT_GELU_, s); }));
            CE_TRY(check_launch(ce::launch_colsum_finish(db1, w.abw, (N1 + 127) / 128, Pd, s), "sparc bwd"));
        } else {
            CE_TRY(tgemm(h, s, "sparc_bwd_dx", w.dvb, Pd, w.W2T, Pd, N1, Pd, Pd, nullptr, 0, nullptr, w.da, true, w.gpart));
            CE_TRY(check_launch(ce::launch_act_bwd_colsum(w.da, w.a, w.da, N1, Pd, ce::ACT_GELU_, db1, w.abw, s), "sparc bwd"));
        }
    }
    CE_TRY(tgemm_tn(h, s, "sparc_bwd_dw", w.da, Pd, w.hv, Dv, Pd, Dv, N1,
                    sp_grad(h, "visual_projection.2.non_linear_projection.0.weight"), w.gpart));
    CE_TRY(tgemm(h, s, "sparc_bwd_dx", w.dvb, Pd, w.WlT, Pd, N1, Dv, Pd, nullptr, 0, nullptr, w.dh, false, w.gpart));
    CE_TRY(tgemm(h, s, "sparc_bwd_dx", w.da, Pd, w.W1T, Pd, N1, Dv, Pd, nullptr, 0, w.dh, w.dh, false, w.gpart));
    CE_TRY(check_launch(ce::launch_ln_grad(w.dh, w.xv, w.stv, N1, Dv, p, 2 * seed, (long)h->sp_sample0 * P,
                                           sp_grad(h, "visual_projection.0.weight"),
                                           sp_grad(h, "visual_projection.0.bias"), w.lng, s), "sparc ln grad"));
    h->sp_state = 1;    // (a new loss_grad is needed before another backward)
    return CE_OK;
}

int ce_apply_rope(ce_handle* h, void* stream, const float* x, int B, int P, int D, float* out) {
    if (!h || !x || !out) return fail(CE_ERR_INVALID, "ce_apply_rope: null argument");
    if (B <= 0 || P <= 0 || D <= 0 || D % 2) return fail(CE_ERR_INVALID, "ce_apply_rope: bad sizes");
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    const float *rc = nullptr, *rs = nullptr;
    if (P == h->G * h->G && D == h->cfg.vision.width) { rc = h->rc_v; rs = h->rs_v; }
    else if (P == h->G * h->G && D == h->cfg.pacl_dim) { rc = h->rc_p; rs = h->rs_p; }
    else return fail(CE_ERR_INVALID, "ce_apply_rope: no RoPE table for P=%d D=%d", P, D);
    return check_launch(ce::launch_rope(out, x, B, P, D, rc, rs, s), "apply_rope");
}

int ce_set_kernel_timing(ce_handle* h, int enable) {
    if (!h) return fail(CE_ERR_INVALID, "ce_set_kernel_timing: null handle");
    DeviceGuard g(h->device);
    CE_TRY(resolve_pending(h));
    h->timing = enable != 0;
    if (enable) {
        h->stats.clear();
        h->stat_idx.clear();
    }
    return CE_OK;
}

int ce_set_kernel_timing_filter(ce_handle* h, const char* tag) {
    if (!h) return fail(CE_ERR_INVALID, "ce_set_kernel_timing_filter: null handle");
    h->timing_only = tag ? tag : "";
    return CE_OK;
}

int ce_kernel_stats(ce_handle* h, int index, char* name, int name_len, double* total_ms, int64_t* launches,
                    double* flops, double* bytes) {
    if (!h) return fail(CE_ERR_INVALID, "ce_kernel_stats: null handle");
    DeviceGuard g(h->device);
    CE_TRY(resolve_pending(h));
    if (index < 0 || index >= (int)h->stats.size()) return fail(CE_ERR_INVALID, "ce_kernel_stats: index out of range");
    const KStat& k = h->stats[index];
    if (name && name_len > 0) {
        strncpy(name, k.name.c_str(), (size_t)name_len - 1);
        name[name_len - 1] = 0;
    }
    if (total_ms) *total_ms = k.ms;
    if (launches) *launches = k.n;
    if (flops) *flops = k.flops;
    if (bytes) *bytes = k.bytes;
    return CE_OK;
}

int ce_kernel_gemm_bf16(void* stream, const void* A, const void* Wt, int M, int N, int K, const float* bias, int act,
                        const float* resid, void* out, int out_dtype) {
    if (!A || !Wt || !out) return fail(CE_ERR_INVALID, "ce_kernel_gemm_bf16: null argument");
    if (M <= 0 || N <= 0 || K <= 0 || K % 64 || N % 64)
        return fail(CE_ERR_INVALID, "ce_kernel_gemm_bf16: need M,N,K > 0, K %% 64 == 0, N %% 64 == 0 (got %d %d %d)", M, N, K);
    if (act < 0 || act > 2 || (out_dtype != CE_F32 && out_dtype != CE_BF16))
        return fail(CE_ERR_INVALID, "ce_kernel_gemm_bf16: bad act/out dtype");
    ce::GemmParams p{};
    p.A = (const bf16_t*)A; p.lda = K; p.W = (const bf16_t*)Wt; p.ldw = K;
    p.M = M; p.N = N; p.K = K; p.bias = bias; p.resid = resid; p.ldr = N; p.out = out; p.ldo = N;
    p.part = ce::gemm_kernel_api_workspace(&p.part_elems);
    return check_launch(ce::launch_gemm(p, act, out_dtype == CE_BF16, (hipStream_t)stream), "gemm");
}

int ce_kernel_gemm_bf16_epi(void* stream, const void* A, const void* Wt, int M, int N, int K, const float* bias,
                            int act, const float* resid, void* out, int out_dtype, int epi, void* xb,
                            void* stats_part, const void* fold_stats, const float* fold_c) {
    if (epi == ce::EPI_PLAIN) return ce_kernel_gemm_bf16(stream, A, Wt, M, N, K, bias, act, resid, out, out_dtype);
    if (!A || !Wt || (!out && epi != ce::EPI_LN_STATS_HL))
        return fail(CE_ERR_INVALID, "ce_kernel_gemm_bf16_epi: null argument");
    if (M <= 0 || N <= 0 || K <= 0 || K % 64 || N % 64)
        return fail(CE_ERR_INVALID, "ce_kernel_gemm_bf16_epi: need M,N,K > 0, K %% 64 == 0, N %% 64 == 0 (got %d %d %d)",
                    M, N, K);
    ce::GemmParams p{};
    p.A = (const bf16_t*)A; p.lda = K; p.W = (const bf16_t*)Wt; p.ldw = K;
    p.M = M; p.N = N; p.K = K; p.bias = bias; p.resid = resid; p.ldr = N; p.out = out; p.ldo = N;
    p.part = ce::gemm_kernel_api_workspace(&p.part_elems);
    if (epi == ce::EPI_LN_STATS) {
        if (act != 0 || !resid || out_dtype != CE_F32 || !xb || !stats_part)
            return fail(CE_ERR_INVALID, "ce_kernel_gemm_bf16_epi: LN stats needs act 0, resid, f32 out, xb, stats_part");
        p.xb = (bf16_t*)xb;
        p.stats_part = (float2*)stats_part;
    } else if (epi == ce::EPI_LN_FOLD) {
        if (act < 0 || act > 2 || resid || out_dtype != CE_BF16 || !bias || !fold_stats || !fold_c)
            return fail(CE_ERR_INVALID, "ce_kernel_gemm_bf16_epi: LN fold needs no resid, bf16 out, bias, fold_stats, fold_c");
        p.fold_stats = (const float2*)fold_stats;
        p.fold_c = fold_c;
    } else if (epi == ce::EPI_LN_STATS_HL || epi == ce::EPI_HL_F32) {
        // residual (and, for 3, output) as hi/lo bf16 planes [2][M][N]
        if (act != 0 || !resid || (epi == ce::EPI_LN_STATS_HL && (!xb || !stats_part)) ||
            (epi == ce::EPI_HL_F32 && out_dtype != CE_F32))
            return fail(CE_ERR_INVALID, "ce_kernel_gemm_bf16_epi: hi/lo epilogues need act 0, resid planes and "
                                        "(3) xb planes + stats_part / (4) f32 out");
        p.resid = nullptr;
        p.rhl = (const bf16_t*)resid;
        p.hl_plane = (long)M * N;
        p.xb = (bf16_t*)xb;
        p.stats_part = (float2*)stats_part;
    } else {
        return fail(CE_ERR_INVALID, "ce_kernel_gemm_bf16_epi: unknown epilogue %d", epi);
    }
    return check_launch(ce::launch_gemm(p, act, out_dtype == CE_BF16, (hipStream_t)stream, epi), "gemm_epi");
}

int ce_kernel_ln_stats_finalize(void* stream, void* stats, const void* part, int rows, int nslab) {
    if (!stats || !part) return fail(CE_ERR_INVALID, "ce_kernel_ln_stats_finalize: null argument");
    if (rows <= 0 || nslab <= 0 || nslab > 64) return fail(CE_ERR_INVALID, "ce_kernel_ln_stats_finalize: bad sizes");
    return check_launch(ce::launch_ln_stats_finalize((float2*)stats, (const float2*)part, rows, nslab, (hipStream_t)stream),
                        "ln_stats_finalize");
}

int ce_set_gemm_auto(int mode) { return ce::set_gemm_auto(mode); }
int ce_set_gemm_variant(int bits) { return ce::set_gemm_variant(bits); }
int ce_set_attn_variant(int var) { return ce::set_attn_variant(var); }
int ce_set_fgemm_variant(int v) { return ce::set_fgemm_variant(v); }
int ce_set_gemm_trace(void* buf, int64_t n_blocks) {
    if (n_blocks < 0) return fail(CE_ERR_INVALID, "ce_set_gemm_trace: negative size");
    ce::set_gemm_trace((unsigned long long*)buf, (long)n_blocks);
    return CE_OK;
}
int ce_gemm_path_counts(int64_t* counts, int n, int reset) {
    if (n > 0 && !counts) return fail(CE_ERR_INVALID, "ce_gemm_path_counts: null counts");
    long long tmp[ce::GEMM_PATH_COUNT];
    ce::gemm_path_counts(tmp, ce::GEMM_PATH_COUNT, reset != 0);
    for (int i = 0; i < n && i < ce::GEMM_PATH_COUNT; ++i) counts[i] = tmp[i];
    return CE_OK;
}
int ce_set_gemm_schedule(int schedule) { return ce::set_gemm_schedule(schedule); }
int ce_set_attn_bwd_variant(int v) { return ce::set_attn_bwd_variant(v); }
int ce_set_train_dw_tn(int on) {
    const int prev = dw_tn() ? 1 : 0;
    g_dw_tn.store(on ? 1 : 0);
    return prev;
}
int ce_set_train_act_bwd_fuse(int on) {
    const int prev = act_bwd_fuse() ? 1 : 0;
    g_act_bwd_fuse.store(on ? 1 : 0);
    return prev;
}
int ce_kernel_gemm_tn_bf16(void* stream, const void* A, int64_t lda, const void* B, int64_t ldb, int M, int N, int K,
                           float* C, int64_t ldc, int scale_rows, float scale) {
    if (!A || !B || !C) return fail(CE_ERR_INVALID, "ce_kernel_gemm_tn_bf16: null argument");
    if (M <= 0 || N <= 0 || K <= 0 || M % 256 || N % 256 || lda < M || ldb < N || ldc < N || lda % 8 || ldb % 8 ||
        ldc % 4)
        return fail(CE_ERR_INVALID, "ce_kernel_gemm_tn_bf16: need M, N multiples of 256, K > 0, lda >= M, ldb >= N, "
                    "ldc >= N (lda, ldb % 8 == 0, ldc % 4 == 0); got M %d N %d K %d", M, N, K);
    ce::TnParams p{};
    p.A = (const bf16_t*)A; p.lda = lda; p.B = (const bf16_t*)B; p.ldb = ldb;
    p.M = M; p.N = N; p.K = K; p.C = C; p.ldc = ldc;
    p.part = ce::gemm_kernel_api_workspace(&p.part_elems);
    p.scale_rows = scale_rows; p.scale = scale;
    return check_launch(ce::launch_gemm_tn(p, (hipStream_t)stream), "gemm_tn");
}
int ce_set_gemm_splitk(int enable) { return ce::set_gemm_splitk(enable); }
int ce_set_ln_fold(ce_handle* h, int enable, int* previous) {
    if (!h) return fail(CE_ERR_INVALID, "ce_set_ln_fold: null handle");
    if (previous) *previous = h->ln_fold ? 1 : 0;
    h->ln_fold = enable != 0;
    return CE_OK;
}

int ce_set_resid_hl(ce_handle* h, int enable, int* previous) {
    if (!h) return fail(CE_ERR_INVALID, "ce_set_resid_hl: null handle");
    if (previous) *previous = h->resid_hl ? 1 : 0;
    h->resid_hl = enable != 0;
    return CE_OK;
}

int ce_set_pooled_prune(ce_handle* h, int enable, int* previous) {
    if (!h) return fail(CE_ERR_INVALID, "ce_set_pooled_prune: null handle");
    if (previous) *previous = h->pooled_prune ? 1 : 0;
    h->pooled_prune = enable != 0;
    return CE_OK;
}

int ce_kernel_attention(void* stream, const void* qkv, void* out, int B, int L, int H, int causal) {
    if (!qkv || !out) return fail(CE_ERR_INVALID, "ce_kernel_attention: null argument");
    if (B <= 0 || L <= 0 || H <= 0) return fail(CE_ERR_INVALID, "ce_kernel_attention: bad sizes");
    return check_launch(ce::launch_attention((const bf16_t*)qkv, (bf16_t*)out, B, L, H, causal != 0, false, (hipStream_t)stream),
                        "attention");
}

int ce_kernel_layernorm(void* stream, const float* in, void* out, int out_dtype, const float* w, const float* b,
                        int rows, int D) {
    if (!in || !out || !w || !b) return fail(CE_ERR_INVALID, "ce_kernel_layernorm: null argument");
    if (rows <= 0 || D <= 0 || D % 256 || D > 1536) return fail(CE_ERR_INVALID, "ce_kernel_layernorm: bad sizes");
    ce::LNParams p{};
    p.in = in; p.ldi = D; p.out = out; p.ldo = D; p.w = w; p.b = b; p.rows = rows; p.D = D;
    return check_launch(ce::launch_layernorm(p, out_dtype == CE_BF16, (hipStream_t)stream), "layernorm");
}

// ---- text-tower training -------------------------------------------------
int ce_train_bind(ce_handle* h, const ce_tensor* params, const ce_tensor* grads, int n) {
    if (!h || (n > 0 && (!params || !grads))) return fail(CE_ERR_INVALID, "ce_train_bind: null argument");
    std::map<std::string, std::pair<float*, float*>> b;
    for (int i = 0; i < n; ++i) {
        if (!params[i].name || !grads[i].name || strcmp(params[i].name, grads[i].name) != 0)
            return fail(CE_ERR_INVALID, "ce_train_bind: entry %d: params and grads must name the same tensor", i);
        const std::string name = canonical(h, params[i].name);
        auto it = h->specs.find(name);
        if (it == h->specs.end()) return fail(CE_ERR_INVALID, "ce_train_bind: unknown tensor '%s'", params[i].name);
        if (params[i].dtype != CE_F32 || grads[i].dtype != CE_F32 || !params[i].data || !grads[i].data)
            return fail(CE_ERR_INVALID, "ce_train_bind: '%s' needs f32 device buffers", params[i].name);
        for (const ce_tensor* t : {&params[i], &grads[i]}) {
            bool ok = t->ndim == (int)it->second.shape.size();
            for (int d = 0; ok && d < t->ndim; ++d) ok = t->shape[d] == it->second.shape[d];
            if (!ok) return fail(CE_ERR_INVALID, "ce_train_bind: '%s' has the wrong shape", params[i].name);
        }
        b[name] = {(float*)params[i].data, (float*)grads[i].data};
    }
    for (const std::string& nm : text_trainable_names(h))
        if (!b.count(nm)) return fail(CE_ERR_INVALID, "ce_train_bind: text tensor '%s' not bound", nm.c_str());
    h->bound = b;
    return CE_OK;
}

int ce_train_sync_weights(ce_handle* h, void* stream) {
    if (!h) return fail(CE_ERR_INVALID, "ce_train_sync_weights: null handle");
    if (h->bound.empty()) return fail(CE_ERR_STATE, "ce_train_sync_weights: no tensors bound (ce_train_bind)");
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    for (auto& kv : h->bound) {
        const WSpec& sp = h->specs.at(kv.first);
        const size_t n = spec_elems(h, kv.first);
        void*& dp = h->dptr[kv.first];
        if (!dp) {
            const size_t bytes = n * (sp.st == ST_BF16 ? 2 : 4);
            if (hipMalloc(&dp, bytes) != hipSuccess) {
                (void)hipGetLastError();
                h->dptr.erase(kv.first);
                return fail(CE_ERR_OOM, "ce_train_sync_weights: cannot allocate '%s'", kv.first.c_str());
            }
        }
        const bool inproj = kv.first.size() > 12 && kv.first.find("attn.in_proj_") != std::string::npos;
        const long row = sp.shape.size() == 2 ? sp.shape[1] : 1;
        const long qrows = inproj ? sp.shape[0] / 3 : 0;
        if (sp.st != ST_BF16 && sp.st != ST_F32)
            return fail(CE_ERR_INVALID, "ce_train_sync_weights: '%s' has an unsupported storage", kv.first.c_str());
        CE_TRY(check_launch(ce::launch_weight_from_master(dp, sp.st == ST_BF16, kv.second.first, (long)n, row, qrows,
                                                          ce::kAttnQScale, s), "weight_from_master"));
        h->loaded[kv.first] = true;
    }
    // the trained tensors' LN folds (host-computed at ce_load_weights) are stale now: encode_text
    // runs the unfolded text blocks until the tower is loaded again
    for (auto& kv : h->folded)
        if (kv.first.rfind("transformer.resblocks.", 0) == 0) kv.second = false;
    return CE_OK;
}

int ce_text_forward_train(ce_handle* h, void* stream, const int64_t* ids, int B, float* out_features) {
    if (!h || !ids) return fail(CE_ERR_INVALID, "ce_text_forward_train: null argument");
    if (B <= 0) return fail(CE_ERR_INVALID, "ce_text_forward_train: batch must be positive");
    if (h->cfg.context_length > 80)
        return fail(CE_ERR_INVALID, "ce_text_forward_train: context %d > 80 (attention backward)", h->cfg.context_length);
    CE_TRY(check_ready(h, false));
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    TrainWs w;
    CE_TRY(train_ws(h, B, w));
    CE_TRY(run_text_train(h, s, w, ids));
    h->tr_B = B;
    if (out_features)
        HIP_TRY(hipMemcpyAsync(out_features, w.f, (size_t)B * w.E * 4, hipMemcpyDeviceToDevice, s));
    return CE_OK;
}

int ce_text_backward(ce_handle* h, void* stream, const float* d_features, int B) {
    if (!h || !d_features) return fail(CE_ERR_INVALID, "ce_text_backward: null argument");
    if (h->bound.empty()) return fail(CE_ERR_STATE, "ce_text_backward: no gradient buffers bound (ce_train_bind)");
    if (B != h->tr_B || B <= 0)
        return fail(CE_ERR_STATE, "ce_text_backward: batch %d does not match the last ce_text_forward_train (%d)", B,
                    h->tr_B);
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    TrainWs w;
    train_layout(h, B, &w, h->tr);
    return run_text_backward(h, s, w, d_features);
}

int ce_text_backward_events(ce_handle* h, void* stream, const float* d_features, int B, void* const* events,
                            int n_events) {
    if (!h || !d_features) return fail(CE_ERR_INVALID, "ce_text_backward_events: null argument");
    if (h->bound.empty()) return fail(CE_ERR_STATE, "ce_text_backward_events: no gradient buffers bound (ce_train_bind)");
    if (B != h->tr_B || B <= 0)
        return fail(CE_ERR_STATE, "ce_text_backward_events: batch %d does not match the last ce_text_forward_train (%d)",
                    B, h->tr_B);
    if (n_events < 0 || (n_events > 0 && !events) || n_events > h->cfg.text.layers + 1)
        return fail(CE_ERR_INVALID, "ce_text_backward_events: %d events for %d blocks (at most layers + 1)", n_events,
                    h->cfg.text.layers);
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    TrainWs w;
    train_layout(h, B, &w, h->tr);
    return run_text_backward(h, s, w, d_features, events, n_events);
}

int ce_contrastive_grad(ce_handle* h, void* stream, const float* A, int Ra, const float* Bm, int Cb, int E, float scale,
                        const int64_t* labels, float weight, float inv_count, float* out2, float* dA, float* dB) {
    if (!h || !A || !Bm || !labels || !out2) return fail(CE_ERR_INVALID, "ce_contrastive_grad: null argument");
    if (Ra <= 0 || Cb <= 0 || E <= 0) return fail(CE_ERR_INVALID, "ce_contrastive_grad: bad sizes");
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    const size_t zR = (size_t)Ra * Cb;
    CE_TRY(ensure_tmp(h, (zR * 2 + 2 * (size_t)Ra + (size_t)std::max(Ra, Cb) * E) * 4));
    float* z = (float*)h->tmp;
    float* zt = z + zR;
    float* rowstat = zt + zR;
    float* acc = rowstat + 2 * (size_t)Ra;
    ce::FGemmParams fp{};       // z = scale * A B^T (ClipLoss logits, loss.py:155-157)
    fp.A = A; fp.lda = E; fp.B = Bm; fp.ldb = E; fp.C = z; fp.ldc = Cb;
    fp.M = Ra; fp.N = Cb; fp.K = E; fp.batch = 1; fp.alpha = scale;
    CE_TRY(check_launch(ce::launch_fgemm(fp, true, s), "logits"));
    CE_TRY(check_launch(ce::launch_ce_grad(z, z, Ra, Cb, labels, weight * inv_count, rowstat, out2, s), "ce_grad"));
    if (dA) {                   // dA += scale * G B
        ce::FGemmParams q{};
        q.A = z; q.lda = Cb; q.B = Bm; q.ldb = E; q.C = acc; q.ldc = E;
        q.M = Ra; q.N = E; q.K = Cb; q.batch = 1; q.alpha = scale;
        CE_TRY(check_launch(ce::launch_fgemm(q, false, s), "dA"));
        CE_TRY(check_launch(ce::launch_axpy(dA, acc, (long)Ra * E, 1.f, s), "axpy"));
    }
    if (dB) {                   // dB += scale * G^T A
        CE_TRY(check_launch(ce::launch_transpose_f32(zt, Ra, z, Cb, Ra, Cb, s), "transpose"));
        ce::FGemmParams q{};
        q.A = zt; q.lda = Ra; q.B = A; q.ldb = E; q.C = acc; q.ldc = E;
        q.M = Cb; q.N = E; q.K = Ra; q.batch = 1; q.alpha = scale;
        CE_TRY(check_launch(ce::launch_fgemm(q, false, s), "dB"));
        CE_TRY(check_launch(ce::launch_axpy(dB, acc, (long)Cb * E, 1.f, s), "axpy"));
    }
    return CE_OK;
}

int ce_adamw(void* stream, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float lr,
             float beta1, float beta2, float eps, float weight_decay, int step) {
    if (n < 0 || (n > 0 && (!param || !grad || !exp_avg || !exp_avg_sq)))
        return fail(CE_ERR_INVALID, "ce_adamw: null argument");
    if (step < 1) return fail(CE_ERR_INVALID, "ce_adamw: step counts from 1 (got %d)", step);
    return check_launch(ce::launch_adamw(param, grad, exp_avg, exp_avg_sq, (long)n, lr, beta1, beta2, eps, weight_decay,
                                         step, (hipStream_t)stream), "adamw");
}

}  // extern "C"
