// codec_records.hip -- exchange records of the MED-PEE side information (the north star's
// "RCCL all-gather of per-slice location maps").
//
// A slice's location map is only meaningful up to candidate `end`, and on real data it is
// almost empty: a bit is set only for an overflow-prone candidate (meta.lm_count of them,
// ~0 on 12-bit CT slices).  So a record carries the map in whichever of two forms is
// shorter for the job:
//   sparse  (meta.lm_count <= 2 * width): the candidate indices of the set bits, ascending,
//           as uint32 (two per word), unused slots zero;
//   dense   (otherwise): map words 0 .. width-1, every bit past `end` zero.
// The map of slice b travels exactly when width >= min(ceil(lm_count / 2), ceil((end+1) / 64)),
// the job-wide max of which the host agrees once and then carries (distributed.py).
// A 2048^2 ct12 slice with 1 KB at T = 2: 72 B per record instead of the ~15.8 KB dense prefix.
//
// Both kernels are one 256-thread workgroup per slice over at most a slice's map prefix:
// latency-sized (a few microseconds per batch), not on the HBM-bound path.
#include "codec_common.h"

namespace {

constexpr int REC_NT = 256;
constexpr int REC_HDR = CODEC_PEE_RECORD_HDR_WORDS;   // codec_pee_meta, in uint64 words

static_assert(sizeof(codec_pee_meta) == REC_HDR * 8, "codec_pee_meta must be 8 words");

__device__ __forceinline__ int dense_words_of(int end, int lm_words) {
    const int dw = (end + 64) >> 6;   // ceil((end + 1) / 64); end >= -1
    return dw < 0 ? 0 : (dw > lm_words ? lm_words : dw);
}

__device__ __forceinline__ u64 end_mask(int end) {   // bits 0 .. end % 64 of end's word
    const int r = end & 63;
    return r == 63 ? ~0ull : ((1ull << (r + 1)) - 1ull);
}

__global__ __launch_bounds__(REC_NT) void k_pee_pack_records(const codec_pee_meta* __restrict__ meta,
                                                              const u64* __restrict__ lm, int lm_words, int width,
                                                              u64* __restrict__ rec) {
    __shared__ uint32_t sh[REC_NT / 64 + 1];
    const int b = blockIdx.x, tid = threadIdx.x;
    const u64* m = reinterpret_cast<const u64*>(meta + b);
    u64* r = rec + (size_t)b * (REC_HDR + width);
    if (tid < REC_HDR) r[tid] = m[tid];
    const int end = meta[b].end, cnt = meta[b].lm_count;
    const int dw = dense_words_of(end, lm_words);
    const u64 last = end_mask(end);
    const u64* row = lm + (size_t)b * lm_words;
    u64* pay = r + REC_HDR;
    if (cnt >= 0 && cnt <= 2 * width) {
        uint32_t* idx = reinterpret_cast<uint32_t*>(pay);
        // every slot zeroed first (the record buffer is reused step to step), then the indices
        for (int s = tid; s < 2 * width; s += REC_NT) idx[s] = 0u;
        __syncthreads();
        uint32_t base = 0;
        for (int w0 = 0; w0 < dw && base < (uint32_t)cnt; w0 += REC_NT) {
            const int w = w0 + tid;
            u64 v = w < dw ? row[w] : 0ull;
            if (w == dw - 1) v &= last;
            uint32_t tot;
            uint32_t pos = base + block_excl_scan<REC_NT>((uint32_t)__popcll(v), sh, &tot);
            while (v) {   // the word's set bits in ascending order
                const int bit = __ffsll((long long)v) - 1;
                if (pos < (uint32_t)cnt) idx[pos] = (uint32_t)(w * 64 + bit);
                ++pos;
                v &= v - 1ull;
            }
            base += tot;
        }
        // fewer set bits in [0, end] than meta.lm_count says (a hand-built meta, an ELOOKBACK
        // slice): the record carries the indices found, its header's lm_count is corrected to
        // their number and flagged, so the receiver decodes exactly that map
        if (base < (uint32_t)cnt && tid == 0) {
            codec_pee_meta* rm = reinterpret_cast<codec_pee_meta*>(r);
            rm->lm_count = (int)base;
            rm->flags |= CODEC_PEE_RECORD_RECOUNTED;
        }
    } else {
        for (int w = tid; w < width; w += REC_NT) {
            u64 v = w < dw ? row[w] : 0ull;
            if (w == dw - 1) v &= last;
            pay[w] = v;
        }
    }
}

__global__ __launch_bounds__(REC_NT) void k_pee_unpack_records(const u64* __restrict__ rec, int width, int lm_cols,
                                                                codec_pee_meta* __restrict__ meta_out,
                                                                u64* __restrict__ lm_out) {
    const int b = blockIdx.x, tid = threadIdx.x;
    const u64* r = rec + (size_t)b * (REC_HDR + width);
    if (meta_out && tid < REC_HDR) reinterpret_cast<u64*>(meta_out + b)[tid] = r[tid];
    if (!lm_out) return;
    const codec_pee_meta* m = reinterpret_cast<const codec_pee_meta*>(r);
    const int cnt = m->lm_count;
    u64* out = lm_out + (size_t)b * lm_cols;
    if (cnt >= 0 && cnt <= 2 * width) {
        const uint32_t* idx = reinterpret_cast<const uint32_t*>(r + REC_HDR);
        for (int w = tid; w < lm_cols; w += REC_NT) {
            const uint32_t lo = (uint32_t)w * 64u;
            int a = 0, z = cnt;   // first index >= lo (the indices are ascending)
            while (a < z) {
                const int mid = (a + z) >> 1;
                if (idx[mid] < lo) a = mid + 1; else z = mid;
            }
            u64 v = 0ull;
            for (int k = a; k < cnt && idx[k] < lo + 64u; ++k) v |= 1ull << (idx[k] & 63u);
            out[w] = v;
        }
    } else {
        const int dw = dense_words_of(m->end, width);
        for (int w = tid; w < lm_cols; w += REC_NT) out[w] = w < dw ? r[REC_HDR + w] : 0ull;
    }
}

}  // namespace

extern "C" {

int codec_pee_pack_records(int32_t B, int32_t lm_words, const codec_pee_meta* meta, const uint64_t* lm,
                           int32_t width, uint64_t* records, void* stream) {
    if (B < 0 || lm_words < 1 || width < 1) return set_err(CODEC_EINVAL, "codec_pee_pack_records: bad sizes");
    if (B == 0) return 0;
    if (!meta || !lm || !records) return set_err(CODEC_EINVAL, "codec_pee_pack_records: NULL pointer argument");
    hipLaunchKernelGGL(k_pee_pack_records, dim3((unsigned)B), dim3(REC_NT), 0, as_stream(stream), meta,
                       reinterpret_cast<const u64*>(lm), (int)lm_words, (int)width, reinterpret_cast<u64*>(records));
    LAUNCH_CHECK("k_pee_pack_records");
    return 0;
}

int codec_pee_unpack_records(int32_t n, int32_t width, const uint64_t* records, int32_t lm_cols,
                             codec_pee_meta* meta_out, uint64_t* lm_out, void* stream) {
    if (n < 0 || width < 1 || lm_cols < 0 || (lm_out && lm_cols < 1))
        return set_err(CODEC_EINVAL, "codec_pee_unpack_records: bad sizes");
    if (n == 0) return 0;
    if (!records || (!meta_out && !lm_out)) return set_err(CODEC_EINVAL, "codec_pee_unpack_records: NULL pointer argument");
    hipLaunchKernelGGL(k_pee_unpack_records, dim3((unsigned)n), dim3(REC_NT), 0, as_stream(stream),
                       reinterpret_cast<const u64*>(records), (int)width, (int)lm_cols, meta_out,
                       reinterpret_cast<u64*>(lm_out));
    LAUNCH_CHECK("k_pee_unpack_records");
    return 0;
}

}  // extern "C"
