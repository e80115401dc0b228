// Host sanitizer check of the C-ABI argument validation ("Host ASan on the C-ABI
// shim").  Linked against a host-only build of the library's translation
// units made with -fsanitize=address,undefined (tests/test_asan_abi.py builds and runs it on
// the CPU box): every codec_* entry is called with NULL pointers, bad shapes, overflowing
// sizes and short workspaces, and must return its negative status (or 0 bytes / a NULL-safe
// value) without touching memory it does not own.  No call here reaches a kernel launch.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "codec_tcc.h"

static int g_fail = 0, g_n = 0;
extern "C" int hip_stub_device_ops(void);   // tests/asan/hip_stubs.cpp

#define EXPECT_NEG(expr)                                                                           \
    do {                                                                                           \
        ++g_n;                                                                                     \
        const long long r_ = (long long)(expr);                                                    \
        if (r_ >= 0) {                                                                             \
            fprintf(stderr, "FAIL line %d: %s returned %lld (want < 0)\n", __LINE__, #expr, r_);   \
            ++g_fail;                                                                              \
        } else if (!codec_last_error() || !codec_last_error()[0]) {                                \
            fprintf(stderr, "FAIL line %d: %s gave no error message\n", __LINE__, #expr);          \
            ++g_fail;                                                                              \
        }                                                                                          \
    } while (0)
#define EXPECT_ZERO(expr)                                                                          \
    do {                                                                                           \
        ++g_n;                                                                                     \
        const long long r_ = (long long)(expr);                                                    \
        if (r_ != 0) {                                                                             \
            fprintf(stderr, "FAIL line %d: %s returned %lld (want 0)\n", __LINE__, #expr, r_);     \
            ++g_fail;                                                                              \
        }                                                                                          \
    } while (0)

static codec_params good_params() {
    codec_params P;
    memset(&P, 0, sizeof(P));
    P.B = 2; P.H = 64; P.W = 64; P.in_bytes = 2; P.out_bytes = 2; P.nbits = 16; P.block = 16;
    P.align = 0; P.mode = CODEC_MODE_HYBRID; P.fixed_s = 0; P.fixed_offset = -1; P.all_mi = 0;
    P.payload_words = 1; P.map_words = 1; P.n_classes = 1; P.beta = 0.4;
    return P;
}

static codec_pee_params good_pee() {
    codec_pee_params P;
    P.B = 2; P.H = 64; P.W = 64; P.bytes = 2; P.T = 2; P.maxval = 65535; P.payload_words = 1;
    P.lm_words = (32 * 32 + 63) / 64;
    return P;
}

// every way a codec_params can be invalid (check_params' rules + overflow extremes)
static std::vector<codec_params> bad_params() {
    std::vector<codec_params> v;
    codec_params P;
    P = good_params(); P.B = 0; v.push_back(P);
    P = good_params(); P.B = -5; v.push_back(P);
    P = good_params(); P.H = 0; v.push_back(P);
    P = good_params(); P.W = -1; v.push_back(P);
    P = good_params(); P.H = 65536; P.W = 65536; v.push_back(P);           // H*W overflows int32
    P = good_params(); P.H = INT32_MAX; P.W = INT32_MAX; v.push_back(P);
    P = good_params(); P.in_bytes = 3; v.push_back(P);
    P = good_params(); P.out_bytes = 0; v.push_back(P);
    P = good_params(); P.nbits = 0; v.push_back(P);
    P = good_params(); P.nbits = 17; v.push_back(P);
    P = good_params(); P.block = 0; v.push_back(P);
    P = good_params(); P.mode = 7; v.push_back(P);
    P = good_params(); P.fixed_s = 17; v.push_back(P);
    P = good_params(); P.fixed_offset = 64 * 64; v.push_back(P);
    P = good_params(); P.fixed_offset = INT32_MAX; v.push_back(P);
    return v;
}

static std::vector<codec_pee_params> bad_pee() {
    std::vector<codec_pee_params> v;
    codec_pee_params P;
    P = good_pee(); P.B = 0; v.push_back(P);
    P = good_pee(); P.B = INT32_MIN; v.push_back(P);
    P = good_pee(); P.H = 0; v.push_back(P);
    P = good_pee(); P.W = -3; v.push_back(P);
    P = good_pee(); P.H = 65536; P.W = 65536; v.push_back(P);
    P = good_pee(); P.bytes = 4; v.push_back(P);
    P = good_pee(); P.T = 0; v.push_back(P);
    P = good_pee(); P.maxval = 0; v.push_back(P);
    P = good_pee(); P.maxval = 65536; v.push_back(P);
    P = good_pee(); P.bytes = 1; P.maxval = 256; v.push_back(P);
    P = good_pee(); P.payload_words = 0; v.push_back(P);
    P = good_pee(); P.lm_words = 0; v.push_back(P);
    P = good_pee(); P.lm_words = 15; v.push_back(P);                        // < nc / 64
    return v;
}

int main() {
    alignas(64) static unsigned char buf[1 << 16];
    void* p = buf;
    const double* lut = reinterpret_cast<const double*>(buf);
    const codec_layout* tab = reinterpret_cast<const codec_layout*>(buf);
    const int32_t* cls = reinterpret_cast<const int32_t*>(buf);
    codec_slice_meta* meta = reinterpret_cast<codec_slice_meta*>(buf);
    uint64_t* w64 = reinterpret_cast<uint64_t*>(buf);
    uint8_t* u8 = buf;
    int32_t* i32 = reinterpret_cast<int32_t*>(buf);
    codec_pee_meta* pmeta = reinterpret_cast<codec_pee_meta*>(buf);

    if (codec_abi_version() != 1) { fprintf(stderr, "FAIL abi version\n"); return 2; }
    if (!codec_last_error()) { fprintf(stderr, "FAIL last_error NULL\n"); return 2; }
    {   // the knobs' tuning switch returns the previous setting (the bad-argument checks below
        // run with it on, so every knob-reading branch is driven too)
        const int was = codec_set_tuning(1);
        if (codec_set_tuning(1) != 1 || (was != 0 && was != 1)) { fprintf(stderr, "FAIL tuning switch\n"); return 2; }
    }

    // ---------------------------------------------------------------- LSB path
    EXPECT_ZERO(codec_workspace_bytes(nullptr));
    for (const codec_params& P : bad_params()) {
        EXPECT_ZERO(codec_workspace_bytes(&P));
        EXPECT_NEG(codec_plan(&P, p, p, lut, 1 << 20, tab, cls, meta, p, 1u << 30, nullptr));
        EXPECT_NEG(codec_encode(&P, p, p, lut, 1 << 20, tab, cls, meta, p, 1u << 30, w64, w64, nullptr));
        EXPECT_NEG(codec_embed(&P, p, p, w64, meta, w64, nullptr));
        EXPECT_NEG(codec_extract(&P, p, w64, meta, p, w64, nullptr));
        EXPECT_NEG(codec_refdecode(&P, p, w64, meta, u8, 16, i32, nullptr));
        EXPECT_NEG(codec_refdecode_dense(&P, p, 0, u8, 4, meta, u8, 16, i32, nullptr));
        EXPECT_NEG(codec_expand_maps(&P, w64, meta, u8, 4, nullptr));
        EXPECT_NEG(codec_restore_dense(&P, p, u8, 4, meta, p, nullptr));
    }
    {
        const codec_params P = good_params();
        const size_t ws = codec_workspace_bytes(&P);
        if (ws == 0) { fprintf(stderr, "FAIL workspace_bytes of good params\n"); ++g_fail; }
        // NULL pointers, one at a time
        EXPECT_NEG(codec_plan(nullptr, p, p, lut, 4096, tab, cls, meta, p, ws, nullptr));
        EXPECT_NEG(codec_plan(&P, nullptr, p, lut, 4096, tab, cls, meta, p, ws, nullptr));
        EXPECT_NEG(codec_plan(&P, p, p, nullptr, 4096, tab, cls, meta, p, ws, nullptr));
        EXPECT_NEG(codec_plan(&P, p, p, lut, 4096, nullptr, cls, meta, p, ws, nullptr));
        EXPECT_NEG(codec_plan(&P, p, p, lut, 4096, tab, nullptr, meta, p, ws, nullptr));
        EXPECT_NEG(codec_plan(&P, p, p, lut, 4096, tab, cls, nullptr, p, ws, nullptr));
        EXPECT_NEG(codec_plan(&P, p, p, lut, 4096, tab, cls, meta, nullptr, ws, nullptr));
        // short workspace / log2 table, no payload classes
        EXPECT_NEG(codec_plan(&P, p, p, lut, 4096, tab, cls, meta, p, ws - 1, nullptr));
        EXPECT_NEG(codec_plan(&P, p, p, lut, 4096, tab, cls, meta, p, 0, nullptr));
        EXPECT_NEG(codec_plan(&P, p, p, lut, 4095, tab, cls, meta, p, ws, nullptr));
        EXPECT_NEG(codec_plan(&P, p, p, lut, -1, tab, cls, meta, p, ws, nullptr));
        codec_params Q = P; Q.n_classes = 0;
        EXPECT_NEG(codec_plan(&Q, p, p, lut, 4096, tab, cls, meta, p, ws, nullptr));
        Q = P; Q.out_bytes = 1;                                               // in place across dtypes
        EXPECT_NEG(codec_plan(&Q, p, p, lut, 4096, tab, cls, meta, p, codec_workspace_bytes(&Q), nullptr));
        // encode / embed / extract pointer and word-count checks
        EXPECT_NEG(codec_encode(&P, p, nullptr, lut, 4096, tab, cls, meta, p, ws, w64, w64, nullptr));
        EXPECT_NEG(codec_encode(&P, p, p, lut, 4096, tab, cls, meta, p, ws, nullptr, w64, nullptr));
        EXPECT_NEG(codec_encode(&P, p, p, lut, 4096, tab, cls, meta, p, ws, w64, nullptr, nullptr));
        EXPECT_NEG(codec_encode(&P, p, buf + 2, lut, 4096, tab, cls, meta, p, ws, w64, w64, nullptr));   // unaligned
        Q = P; Q.payload_words = 0;
        EXPECT_NEG(codec_encode(&Q, p, p, lut, 4096, tab, cls, meta, p, ws, w64, w64, nullptr));
        Q = P; Q.map_words = -1;
        EXPECT_NEG(codec_embed(&Q, p, p, w64, meta, w64, nullptr));
        EXPECT_NEG(codec_embed(&P, nullptr, p, w64, meta, w64, nullptr));
        EXPECT_NEG(codec_embed(&P, p, buf + 1, w64, meta, w64, nullptr));
        EXPECT_NEG(codec_embed(&P, p, p, nullptr, meta, w64, nullptr));
        EXPECT_NEG(codec_embed(&P, p, p, w64, nullptr, w64, nullptr));
        EXPECT_NEG(codec_embed(&P, p, p, w64, meta, nullptr, nullptr));
        EXPECT_NEG(codec_extract(&P, nullptr, w64, meta, p, w64, nullptr));
        EXPECT_NEG(codec_extract(&P, p, nullptr, meta, p, w64, nullptr));
        EXPECT_NEG(codec_extract(&P, p, w64, nullptr, p, w64, nullptr));
        Q = P; Q.out_bytes = 1;
        EXPECT_NEG(codec_extract(&Q, p, w64, meta, p, w64, nullptr));
        Q = P; Q.payload_words = 0;
        EXPECT_NEG(codec_extract(&Q, p, w64, meta, p, w64, nullptr));
        // reference-layout conversions
        EXPECT_NEG(codec_refdecode(&P, p, w64, meta, u8, 0, i32, nullptr));
        EXPECT_NEG(codec_refdecode(&P, p, w64, meta, nullptr, 16, i32, nullptr));
        EXPECT_NEG(codec_refdecode(&P, p, w64, meta, u8, 16, nullptr, nullptr));
        EXPECT_NEG(codec_refdecode_dense(&P, p, 0, u8, 0, meta, u8, 16, i32, nullptr));
        EXPECT_NEG(codec_refdecode_dense(&P, p, 0, u8, 17, meta, u8, 16, i32, nullptr));
        EXPECT_NEG(codec_refdecode_dense(&P, p, 1, nullptr, 4, meta, u8, 16, i32, nullptr));
        EXPECT_NEG(codec_expand_maps(&P, w64, meta, u8, 0, nullptr));
        EXPECT_NEG(codec_expand_maps(&P, nullptr, meta, u8, 4, nullptr));
        EXPECT_NEG(codec_restore_dense(&P, p, u8, 17, meta, p, nullptr));
        EXPECT_NEG(codec_restore_dense(&P, p, u8, 4, meta, nullptr, nullptr));
        EXPECT_NEG(codec_unpack_planes(nullptr, p, 0, 1, p, 1, nullptr));
        EXPECT_NEG(codec_unpack_planes(&P, p, -1, 1, p, 1, nullptr));
        EXPECT_NEG(codec_unpack_planes(&P, p, 0, 0, p, 1, nullptr));
        EXPECT_NEG(codec_unpack_planes(&P, p, 0, 1, p, 3, nullptr));
        EXPECT_NEG(codec_unpack_planes(&P, nullptr, 0, 1, p, 1, nullptr));
        EXPECT_NEG(codec_merge_planes(nullptr, p, 1, 1, p, nullptr));
        EXPECT_NEG(codec_merge_planes(&P, p, 0, 1, p, nullptr));
        EXPECT_NEG(codec_merge_planes(&P, p, 1, 4, p, nullptr));
        EXPECT_NEG(codec_merge_planes(&P, p, 1, 1, nullptr, nullptr));
        Q = P; Q.B = 0;
        EXPECT_NEG(codec_unpack_planes(&Q, p, 0, 1, p, 1, nullptr));
        EXPECT_NEG(codec_merge_planes(&Q, p, 1, 1, p, nullptr));
    }
    // lsb_embed_block_adaptive pieces
    EXPECT_NEG(codec_block_variance(0, 8, 8, 1, 4, p, reinterpret_cast<double*>(buf), nullptr));
    EXPECT_NEG(codec_block_variance(1, 8, 8, 3, 4, p, reinterpret_cast<double*>(buf), nullptr));
    EXPECT_NEG(codec_block_variance(1, 8, 8, 1, 0, p, reinterpret_cast<double*>(buf), nullptr));
    EXPECT_NEG(codec_block_variance(1, 8, 8, 1, 65536, p, reinterpret_cast<double*>(buf), nullptr));
    EXPECT_NEG(codec_block_variance(INT32_MAX, INT32_MAX, INT32_MAX, 1, 1, p, reinterpret_cast<double*>(buf), nullptr));
    EXPECT_NEG(codec_block_variance(1, 8, 8, 1, 4, nullptr, reinterpret_cast<double*>(buf), nullptr));
    EXPECT_NEG(codec_block_variance(1, 8, 8, 1, 4, p, nullptr, nullptr));
    const int64_t runs[4] = {0, 0, 1, 0};
    EXPECT_NEG(codec_lsb_runs(0, 64, 1, p, u8, u8, 64, runs, 1, nullptr));
    EXPECT_NEG(codec_lsb_runs(1, 0, 1, p, u8, u8, 64, runs, 1, nullptr));
    EXPECT_NEG(codec_lsb_runs(1, 64, 4, p, u8, u8, 64, runs, 1, nullptr));
    EXPECT_NEG(codec_lsb_runs(1, 64, 1, nullptr, u8, u8, 64, runs, 1, nullptr));
    EXPECT_NEG(codec_lsb_runs(1, 64, 1, p, nullptr, u8, 64, runs, 1, nullptr));
    EXPECT_NEG(codec_lsb_runs(1, 64, 1, p, u8, u8, -1, runs, 1, nullptr));
    EXPECT_NEG(codec_lsb_runs(1, 64, 1, p, u8, u8, 64, runs, -1, nullptr));
    EXPECT_NEG(codec_lsb_runs(1, 64, 1, p, u8, nullptr, 64, runs, 1, nullptr));
    EXPECT_NEG(codec_lsb_runs(1, 64, 1, p, u8, u8, 64, nullptr, 1, nullptr));
    EXPECT_ZERO(codec_lsb_runs(1, 64, 1, p, u8, nullptr, 64, nullptr, 0, nullptr));   // nothing to do

    // ---------------------------------------------------------------- MED-PEE
    EXPECT_ZERO(codec_pee_workspace_bytes(nullptr));
    EXPECT_ZERO(codec_pee_extract_flag_offset(nullptr));
    EXPECT_ZERO(codec_pee_diag_offset(nullptr));
    for (const codec_pee_params& P : bad_pee()) {
        EXPECT_ZERO(codec_pee_workspace_bytes(&P));
        EXPECT_ZERO(codec_pee_extract_flag_offset(&P));
        EXPECT_ZERO(codec_pee_diag_offset(&P));
        EXPECT_NEG(codec_pee_reset(&P, p, 1u << 30, nullptr));
        EXPECT_NEG(codec_pee_embed(&P, p, p, w64, i32, pmeta, w64, p, 1u << 30, nullptr));
        EXPECT_NEG(codec_pee_embed_ts(&P, p, p, w64, i32, i32, pmeta, w64, p, 1u << 30, nullptr));
        EXPECT_NEG(codec_pee_capacity(&P, p, 4, i32, i32, i32, p, 1u << 30, nullptr));
        EXPECT_NEG(codec_pee_embed_auto(&P, p, p, w64, i32, 4, i32, pmeta, w64, p, 1u << 30, nullptr));
        EXPECT_NEG(codec_pee_extract(&P, p, pmeta, w64, p, w64, p, 1u << 30, nullptr));
        EXPECT_NEG(codec_pee_multi_embed_pass(&P, 0, p, p, w64, i32, pmeta, w64, p, 1u << 30, nullptr));
        EXPECT_NEG(codec_pee_multi_extract_pass(&P, 0, p, pmeta, w64, p, w64, p, 1u << 30, nullptr));
        EXPECT_NEG(codec_pee_multi_embed(&P, p, p, w64, i32, pmeta, w64, p, 1u << 30, nullptr));
        EXPECT_NEG(codec_pee_multi_extract(&P, p, pmeta, w64, p, w64, p, 1u << 30, nullptr));
    }
    {
        const codec_pee_params P = good_pee();
        const size_t ws = codec_pee_workspace_bytes(&P);
        if (ws == 0) { fprintf(stderr, "FAIL pee workspace_bytes of good params\n"); ++g_fail; }
        EXPECT_NEG(codec_pee_embed(&P, nullptr, p, w64, i32, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_embed(&P, p, nullptr, w64, i32, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_embed(&P, p, p, nullptr, i32, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_embed(&P, p, p, w64, nullptr, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_embed(&P, p, p, w64, i32, nullptr, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_embed(&P, p, p, w64, i32, pmeta, nullptr, p, ws, nullptr));
        EXPECT_NEG(codec_pee_embed(&P, p, p, w64, i32, pmeta, w64, nullptr, ws, nullptr));
        EXPECT_NEG(codec_pee_embed(&P, p, p, w64, i32, pmeta, w64, p, ws - 1, nullptr));
        EXPECT_NEG(codec_pee_embed(&P, p, p, w64, i32, pmeta, w64, p, 0, nullptr));
        EXPECT_NEG(codec_pee_embed_ts(&P, p, p, w64, i32, i32, pmeta, w64, p, ws - 8, nullptr));
        EXPECT_NEG(codec_pee_capacity(&P, nullptr, 4, i32, i32, i32, p, ws, nullptr));
        EXPECT_NEG(codec_pee_capacity(&P, p, 0, i32, i32, i32, p, ws, nullptr));
        EXPECT_NEG(codec_pee_capacity(&P, p, 65, i32, i32, i32, p, ws, nullptr));
        EXPECT_NEG(codec_pee_capacity(&P, p, 4, nullptr, i32, i32, p, ws, nullptr));   // t_out needs lengths
        EXPECT_NEG(codec_pee_capacity(&P, p, 4, i32, i32, i32, nullptr, ws, nullptr));
        EXPECT_NEG(codec_pee_capacity(&P, p, 4, i32, i32, i32, p, ws - 1, nullptr));
        EXPECT_NEG(codec_pee_embed_auto(&P, p, p, w64, i32, 0, i32, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_embed_auto(&P, p, p, w64, i32, 65, i32, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_embed_auto(&P, p, p, w64, i32, 4, nullptr, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_embed_auto(&P, p, p, w64, i32, 4, i32, pmeta, w64, p, ws - 1, nullptr));
        EXPECT_NEG(codec_pee_extract(&P, nullptr, pmeta, w64, p, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_extract(&P, p, nullptr, w64, p, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_extract(&P, p, pmeta, nullptr, p, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_extract(&P, p, pmeta, w64, nullptr, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_extract(&P, p, pmeta, w64, p, nullptr, p, ws, nullptr));
        EXPECT_NEG(codec_pee_extract(&P, p, pmeta, w64, p, w64, nullptr, ws, nullptr));
        EXPECT_NEG(codec_pee_extract(&P, p, pmeta, w64, p, w64, p, ws - 1, nullptr));
        EXPECT_NEG(codec_pee_multi_embed_pass(&P, -1, p, p, w64, i32, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_embed_pass(&P, 4, p, p, w64, i32, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_embed_pass(&P, 1, nullptr, p, w64, i32, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_embed_pass(&P, 1, p, nullptr, w64, i32, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_embed_pass(&P, 1, p, p, nullptr, i32, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_embed_pass(&P, 1, p, p, w64, nullptr, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_embed_pass(&P, 1, p, p, w64, i32, nullptr, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_embed_pass(&P, 1, p, p, w64, i32, pmeta, nullptr, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_embed_pass(&P, 1, p, p, w64, i32, pmeta, w64, nullptr, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_embed_pass(&P, 1, p, p, w64, i32, pmeta, w64, p, ws - 1, nullptr));
        EXPECT_NEG(codec_pee_multi_extract_pass(&P, 5, p, pmeta, w64, p, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_extract_pass(&P, 2, nullptr, pmeta, w64, p, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_extract_pass(&P, 2, p, nullptr, w64, p, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_extract_pass(&P, 2, p, pmeta, nullptr, p, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_extract_pass(&P, 2, p, pmeta, w64, nullptr, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_extract_pass(&P, 2, p, pmeta, w64, p, nullptr, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_extract_pass(&P, 2, p, pmeta, w64, p, w64, nullptr, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_extract_pass(&P, 2, p, pmeta, w64, p, w64, p, ws - 1, nullptr));
        EXPECT_NEG(codec_pee_multi_embed(&P, nullptr, p, w64, i32, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_embed(&P, p, nullptr, w64, i32, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_embed(&P, p, p, nullptr, i32, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_embed(&P, p, p, w64, nullptr, pmeta, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_embed(&P, p, p, w64, i32, nullptr, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_embed(&P, p, p, w64, i32, pmeta, nullptr, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_embed(&P, p, p, w64, i32, pmeta, w64, nullptr, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_embed(&P, p, p, w64, i32, pmeta, w64, p, ws - 1, nullptr));
        EXPECT_NEG(codec_pee_multi_extract(&P, nullptr, pmeta, w64, p, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_extract(&P, p, nullptr, w64, p, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_extract(&P, p, pmeta, nullptr, p, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_extract(&P, p, pmeta, w64, nullptr, w64, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_extract(&P, p, pmeta, w64, p, nullptr, p, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_extract(&P, p, pmeta, w64, p, w64, nullptr, ws, nullptr));
        EXPECT_NEG(codec_pee_multi_extract(&P, p, pmeta, w64, p, w64, p, ws - 1, nullptr));
        EXPECT_NEG(codec_pee_reset(nullptr, p, ws, nullptr));
        EXPECT_NEG(codec_pee_reset(&P, nullptr, ws, nullptr));
        EXPECT_NEG(codec_pee_reset(&P, p, ws - 1, nullptr));
    }
    // exchange records
    EXPECT_NEG(codec_pee_pack_records(-1, 4, pmeta, w64, 1, w64, nullptr));
    EXPECT_NEG(codec_pee_pack_records(2, 0, pmeta, w64, 1, w64, nullptr));
    EXPECT_NEG(codec_pee_pack_records(2, 4, pmeta, w64, 0, w64, nullptr));
    EXPECT_NEG(codec_pee_pack_records(2, 4, nullptr, w64, 1, w64, nullptr));
    EXPECT_NEG(codec_pee_pack_records(2, 4, pmeta, nullptr, 1, w64, nullptr));
    EXPECT_NEG(codec_pee_pack_records(2, 4, pmeta, w64, 1, nullptr, nullptr));
    EXPECT_ZERO(codec_pee_pack_records(0, 4, nullptr, nullptr, 1, nullptr, nullptr));
    EXPECT_NEG(codec_pee_unpack_records(-1, 1, w64, 4, pmeta, w64, nullptr));
    EXPECT_NEG(codec_pee_unpack_records(2, 0, w64, 4, pmeta, w64, nullptr));
    EXPECT_NEG(codec_pee_unpack_records(2, 1, w64, 0, pmeta, w64, nullptr));
    EXPECT_NEG(codec_pee_unpack_records(2, 1, w64, -1, pmeta, nullptr, nullptr));
    EXPECT_NEG(codec_pee_unpack_records(2, 1, nullptr, 4, pmeta, w64, nullptr));
    EXPECT_NEG(codec_pee_unpack_records(2, 1, w64, 4, nullptr, nullptr, nullptr));
    EXPECT_ZERO(codec_pee_unpack_records(0, 1, nullptr, 4, nullptr, nullptr, nullptr));

    // quality moments, profiling window, diagnostics
    EXPECT_NEG(codec_quality_moments(0, 8, 8, 2, p, p, w64, nullptr));
    EXPECT_NEG(codec_quality_moments(1, -8, 8, 2, p, p, w64, nullptr));
    EXPECT_NEG(codec_quality_moments(1, 8, 8, 3, p, p, w64, nullptr));
    EXPECT_NEG(codec_quality_moments(1, 65536, 65536, 2, p, p, w64, nullptr));
    EXPECT_NEG(codec_quality_moments(1, 8, 8, 2, nullptr, p, w64, nullptr));
    EXPECT_NEG(codec_quality_moments(1, 8, 8, 2, p, nullptr, w64, nullptr));
    EXPECT_NEG(codec_quality_moments(1, 8, 8, 2, p, p, nullptr, nullptr));
    EXPECT_NEG(codec_profile_begin(0));
    EXPECT_NEG(codec_profile_begin(-4));
    EXPECT_NEG(codec_profile_end(reinterpret_cast<float*>(buf), i32, 16));      // no window open
    EXPECT_NEG(codec_debug_res_trace(nullptr, 16));
    EXPECT_NEG(codec_debug_res_trace(reinterpret_cast<unsigned long long*>(buf), -1));

    if (!codec_build_digest()) { fprintf(stderr, "FAIL build digest NULL\n"); ++g_fail; }
    if (hip_stub_device_ops() != 0) {
        fprintf(stderr, "FAIL %d launches / memory operations reached the runtime\n", hip_stub_device_ops());
        ++g_fail;
    }
    printf("abi_args: %d calls, %d failures\n", g_n, g_fail);
    return g_fail ? 1 : 0;
}
