/*
 * codec_tcc.h -- C ABI of libcodec_hip.so, the MI355X (gfx950) implementation of the
 * reference's LSB bit-plane embed/extract pixel path (wesleyfn/codec-tcc, src/codec.py).
 *
 * Boundary contract (mirrors the reference's Python function boundary):
 *   - every pointer argument is a DEVICE pointer owned by the caller (torch tensors);
 *     `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream);
 *   - every call is asynchronous on `stream` and thread-safe given distinct streams and
 *     buffers; nothing is allocated inside (workspace is caller-provided).  A workspace is
 *     one of those buffers: calls that share one are ordered on one stream, since some
 *     carry state from call to call in it (codec_pee_workspace_bytes states the recovery
 *     rules: shape changes are detected and re-zeroed, stale state is never read as valid,
 *     codec_pee_reset after a failed call);
 *   - return value: 0 on success, < 0 on error (argument error or negated hipError_t);
 *     codec_last_error() returns a thread-local message.  The Python host layer turns a
 *     non-zero status into an exception, as the reference raises ValueError (codec.py:34-37).
 *
 * Pixel layout in HBM: a batch of B slices, each H x W row-major, slices contiguous
 * ([B][H][W]), uint8 or uint16 little-endian.  Location maps and payloads are packed
 * bitstrings, LSB-first inside uint64 words, one fixed-size row of words per slice.
 */
#ifndef CODEC_TCC_H
#define CODEC_TCC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CODEC_ABI_VERSION 1
#define CODEC_MAX_PLANES 16

/* Embedder variants (reference functions they reproduce). */
#define CODEC_MODE_HYBRID 0 /* lsb_embed_block_then_multiplane, codec.py:412-487 */
#define CODEC_MODE_MULTI 1  /* lsb_embed_multi_plane,           codec.py:276-318 */

/* codec_slice_meta.flags */
#define CODEC_FLAG_OVERLAP 1u   /* windows of different planes may share pixels   */
#define CODEC_FLAG_LOSSY 2u     /* segments do not tile the payload (T < s, clamp) */
#define CODEC_FLAG_BADLUT 4u    /* log2 table shorter than H*W (status error)      */
#define CODEC_FLAG_DECIDE_TIMEOUT 8u /* split decision: a plane workgroup never reported (status 2) */
/* The s decision is guard-banded.  Since every bit plane X is a function of the
 * image Y, I(X;Y) = H(X) exactly, and the reference's MI (codec.py:554) differs from H(X) only
 * by the rounding of its numpy-order sums (~1e-13 at most).  Unless all_mi is set, s is
 * decided from the cumulative H(X) against beta * H(Y) when every prefix of that walk lies
 * more than 1e-9 from its target -- the same s as the reference's loop -- and the slice
 * records CODEC_FLAG_INFO_FAST: mi[] holds H(X) of the planes the loop evaluated and cum_info
 * their sum (entropy and target stay numpy-exact).  A slice with a prefix inside the band is
 * decided by the exact numpy-order sums (mi[], cum_info exact) and records
 * CODEC_FLAG_GUARD_FALLBACK.  all_mi = 1 always takes the exact sums. */
#define CODEC_FLAG_INFO_FAST 16u
#define CODEC_FLAG_GUARD_FALLBACK 32u

/* Call parameters (one batch: all slices share shape and dtype). */
typedef struct codec_params {
    int32_t B, H, W;
    int32_t in_bytes;      /* cover dtype: 1 = uint8, 2 = uint16                         */
    int32_t out_bytes;     /* stego dtype: merge_modalities rule, codec.py:221           */
    int32_t nbits;         /* bit planes examined, codec.py:567 (1..16)                  */
    int32_t block;         /* search_block_size, codec.py:412,435 (>= 1)                 */
    int32_t align;         /* align_across_planes, codec.py:412,484                      */
    int32_t mode;          /* CODEC_MODE_*                                               */
    int32_t fixed_s;       /* > 0: use this s instead of the decision (codec.py:584-593) */
    int32_t fixed_offset;  /* >= 0: use this start offset instead of the block search    */
    int32_t all_mi;        /* 1: evaluate MI of every plane (diagnostics), s unchanged   */
    int32_t payload_words; /* uint64 words per slice in payload buffers                  */
    int32_t map_words;     /* uint64 words per slice in location-map buffers             */
    int32_t n_classes;     /* rows of the layout table / 16                              */
    int32_t reserved;
    double beta;           /* retention target, codec.py:561,575                         */
} codec_params;

/* Segment plan for one (payload length T, plane count s), built on the host by the
 * reference's own rule (distribute_message_segments, codec.py:242-274). Indexed by
 * destination plane p except perm, which is the segment order (segment_indices). */
typedef struct codec_layout {
    int32_t sizes[CODEC_MAX_PLANES]; /* distributed_sizes[p]  (codec.py:253-259)          */
    int32_t perm[CODEC_MAX_PLANES];  /* segment_indices[j]    (codec.py:262-264)          */
    int32_t src[CODEC_MAX_PLANES];   /* first payload bit of plane p's segment (slice)    */
    int32_t len[CODEC_MAX_PLANES];   /* len(segment) of plane p (python slice semantics) */
} codec_layout;

/* Per-slice result record (fixed size; this is what the multi-GPU path all-gathers). */
typedef struct codec_slice_meta {
    int32_t s;            /* number of local planes                                  */
    int32_t start_offset; /* raster offset of the best block, codec.py:453          */
    int32_t total_used;   /* sum of embedded bits, codec.py:480                      */
    uint32_t flags;       /* CODEC_FLAG_*                                            */
    int32_t npix;         /* H*W                                                     */
    int32_t nbits;
    int32_t status;       /* 0 ok                                                    */
    int32_t nonzero_bins; /* distinct pixel values                                   */
    int32_t perm[CODEC_MAX_PLANES];  /* segment_indices                             */
    int32_t sizes[CODEC_MAX_PLANES]; /* segments_lengths as the reference returns them */
    int32_t n[CODEC_MAX_PLANES];     /* bits embedded in plane p (window length)     */
    int32_t src[CODEC_MAX_PLANES];   /* payload bit index of plane p's first bit     */
    int32_t off[CODEC_MAX_PLANES];   /* raster start of plane p's window             */
    int32_t cat[CODEC_MAX_PLANES];   /* position of plane p's bits in the location map */
    double entropy;       /* calculate_entropy(cover), bit-exact (codec.py:489-502)  */
    double target;        /* beta * entropy                                          */
    double cum_info;      /* cumulative MI at the decision                           */
    int32_t span_lo;      /* every window lies in the circular pixel interval          */
    int32_t span_len;     /*   [span_lo, span_lo + span_len) mod H*W                   */
    double mi[CODEC_MAX_PLANES]; /* calculate_mutual_information per plane, evaluated ones */
} codec_slice_meta;

int codec_abi_version(void);
const char* codec_last_error(void);
/* Tuning switch of the A/B knobs.  Every launch-shape choice (scan sweep, ring depths, store
 * policy, decision path, ...) has a measured default.  The CODEC_* environment variables that
 * override them are honoured only while this switch is on: CODEC_TUNING=1 in the
 * environment when the library is loaded (read once), or codec_set_tuning(1).  With it off --
 * the default -- no call reads the environment.  The fault-injection knobs additionally need
 * CODEC_DEBUG=1.  Returns the previous setting.  No reference counterpart. */
int codec_set_tuning(int32_t on);
/* SHA-256 (hex) of the sources, headers and compiler flags this library was built from
 * (codec_tcc_amd/build.py); the Python loader refuses an in-tree library whose digest differs
 * from the tree's.  No reference counterpart (build integrity only). */
const char* codec_build_digest(void);

/* Bytes of scratch `codec_plan` needs for these parameters.  Zero-initialise the workspace
 * once before its first use: codec_plan / codec_encode expect its histogram words clear and
 * leave them clear (the decision kernel zeroes what the scan wrote), so no call memsets it
 * (env CODEC_HIST_MEMSET=1 restores a per-call memset).  A call that fails after launching
 * the scan re-clears it on the stream. */
size_t codec_workspace_bytes(const codec_params* P);

/* Decomposition + block search + segment plan, and the cover->stego copy:
 *   replaces adaptive_modalities_decomposition (codec.py:561-599, incl. calculate_entropy
 *   :489-502 and calculate_mutual_information :504-559), the block-variance search of
 *   lsb_embed_block_then_multiplane (codec.py:431-453) and the merge of untouched planes
 *   (merge_modalities, codec.py:215-237).
 * cover[B][H][W] (in_bytes) -> stego[B][H][W] (out_bytes; may be NULL: plan only),
 * meta[B].  log2_lut[c-1] = numpy.log2(c / (H*W)) for c = 1..H*W (lut_len >= H*W);
 * table[n_classes*16 + (s-1)] is the layout for payload class slice_class[b] and s.
 * stego == cover (same dtype) = in place: the pass only reads, codec_embed then rewrites
 * the window pixels of the cover buffer itself. */
int codec_plan(const codec_params* P, const void* cover, void* stego, const double* log2_lut,
               int64_t lut_len, const codec_layout* table, const int32_t* slice_class,
               codec_slice_meta* meta, void* workspace, size_t workspace_bytes, void* stream);

/* codec_plan + codec_embed in one call, same results: when stego and cover share a dtype the
 * decision kernel embeds each slice's payload itself once its windows are known (one launch
 * fewer, and the embed runs inside the decision's workgroup); otherwise plan then embed.
 * (Batched API: Codec.encode.) */
int codec_encode(const codec_params* P, const void* cover, void* stego, const double* log2_lut,
                 int64_t lut_len, const codec_layout* table, const int32_t* slice_class,
                 codec_slice_meta* meta, void* workspace, size_t workspace_bytes,
                 const uint64_t* payload, uint64_t* maps, void* stream);

/* Window writes + location map: the embed loop of lsb_embed_block_then_multiplane
 * (codec.py:455-485) / lsb_embed_multi_plane (codec.py:288-316).  stego must already
 * hold the copy written by codec_plan.  payload[B][payload_words] (bit b of slice =
 * message bit b), maps[B][map_words] receives bit j = (cover bit ^ message bit) of the
 * j-th embedded bit in segment order (the non-zero region of the reference bitmaps). */
int codec_embed(const codec_params* P, const void* cover, void* stego, const uint64_t* payload,
                const codec_slice_meta* meta, uint64_t* maps, void* stream);

/* True extraction: payload bits in segment order + cover restore (inverse of the above).
 * cover_out may be NULL (payload only).  payload_out[B][payload_words].
 * cover_out == stego = in place: only the window pixels are rewritten (after the gather). */
int codec_extract(const codec_params* P, const void* stego, const uint64_t* maps,
                  const codec_slice_meta* meta, void* cover_out, uint64_t* payload_out,
                  void* stream);

/* decode_message (codec.py:752-787) bit stream, from the packed location maps: per plane
 * the stego LSBs at the first segments_lengths[p] flipped positions in ascending raster
 * order, planes concatenated in index order.  bits_out[B][bits_cap] one byte per bit,
 * counts_out[B] = number of bits written. */
int codec_refdecode(const codec_params* P, const void* stego, const uint64_t* maps,
                    const codec_slice_meta* meta, uint8_t* bits_out, int32_t bits_cap,
                    int32_t* counts_out, void* stream);

/* decode_message from DENSE reference bitmaps (codec.py:767-772 on np.split blobs,
 * codec.py:820-821).  src is either the stego image (src_is_planes = 0; plane p is bit p)
 * or stacked planes [B][smax][H*W] of dtype in_bytes (src_is_planes = 1; value & 1).
 * dense[B][smax][H*W] uint8.  meta supplies s, perm and sizes (segments_lengths).
 * counts_out must hold B*17 int32: [0,B) bits written per slice, the rest is scratch. */
int codec_refdecode_dense(const codec_params* P, const void* src, int32_t src_is_planes,
                          const uint8_t* dense, int32_t smax, const codec_slice_meta* meta,
                          uint8_t* bits_out, int32_t bits_cap, int32_t* counts_out, void* stream);

/* Dense reference bitmaps from packed maps: dense[B][smax][H*W] uint8 (codec.py:462-476,
 * np.stack at codec.py:888).  Planes >= s are zero. */
int codec_expand_maps(const codec_params* P, const uint64_t* maps, const codec_slice_meta* meta,
                      uint8_t* dense, int32_t smax, void* stream);

/* Cover restore from DENSE bitmaps: cover = stego ^ sum_p (dense[p] & 1) << p, p < s. */
int codec_restore_dense(const codec_params* P, const void* stego, const uint8_t* dense,
                        int32_t smax, const codec_slice_meta* meta, void* cover_out,
                        void* stream);

/* Bit-plane unpack, (img >> i) & 1 in the image dtype for i in [first, first+count):
 * codec.py:571 and extract_local_planes codec.py:789-793.  planes[B][count][H*W]. */
int codec_unpack_planes(const codec_params* P, const void* img, int32_t first, int32_t count,
                        void* planes, int32_t plane_bytes, void* stream);

/* merge_modalities (codec.py:215-237): out = OR_k (out_t)(planes[k]) << k, k < nplanes,
 * planes stacked LSB-first [B][nplanes][H*W] of plane_bytes each. */
int codec_merge_planes(const codec_params* P, const void* planes, int32_t nplanes,
                       int32_t plane_bytes, void* out, void* stream);

/* ---- lsb_embed_block_adaptive (codec.py:320-410).
 * Step 1 (codec.py:349-358): scores[b][by*nbx+bx] = float(np.var(block)) of every
 * block x block tile (partial at the right/bottom edges) of each of the B planes, planes
 * [B][H][W] of `bytes` holding 0/1 values, numpy-exact (pairwise float64 order). */
int codec_block_variance(int32_t B, int32_t H, int32_t W, int32_t bytes, int32_t block, const void* planes,
                         double* scores, void* stream);
/* Step 2 (codec.py:372-404), after the host's stable descending sort of each plane's
 * scores and its walk of the blocks: runs[r] = {plane, first pixel, length, first bit}
 * (int64 x 4, device).  planes[p][off+i] := (old & 0xFE) | bits[p*bits_stride+src+i],
 * bitmaps[p][off+i] := old ^ new, for i < length.  Runs must not overlap. */
int codec_lsb_runs(int32_t nplanes, int64_t npx, int32_t bytes, void* planes, uint8_t* bitmaps, const uint8_t* bits,
                   int64_t bits_stride, const int64_t* runs, int32_t nruns, void* stream);

/* ---- MED-predictor prediction-error expansion (the north star's PEE).
 * Not present in the reference: this build's own scheme, specified in
 * oracle/pee_cpu.py (parity unpinned; checked bit-exact against that spec and by
 * reversibility).  Candidates are the (odd, odd) sublattice, whose MED neighbours are
 * never modified; bit j goes to the j-th expandable candidate (-T <= e < T) in raster
 * order, others up to `end` are shifted by T, overflow-prone ones are skipped and set in
 * the location map lm (one bit per candidate index). */
typedef struct codec_pee_params {
    int32_t B, H, W;
    int32_t bytes;         /* 1 = uint8, 2 = uint16                                   */
    int32_t T;             /* expansion threshold (>= 1)                              */
    int32_t maxval;        /* largest admissible pixel value (overflow bound)         */
    int32_t payload_words; /* uint64 words per slice in payload buffers               */
    int32_t lm_words;      /* uint64 words per slice of the location map (>= nc/64)   */
} codec_pee_params;

typedef struct codec_pee_meta {
    int32_t T, maxval, L, end; /* end = last processed candidate index, -1 if none */
    int32_t nc, ntiles, tile_end, status; /* status 1: payload exceeds capacity    */
    int32_t capacity, lm_count, h, w;
    int32_t flags;             /* CODEC_PEE_PARTIAL                                 */
    int32_t reserved[3];
} codec_pee_meta;

/* meta.flags: the single-pass embed (the default wherever W % 8 == 0 and the buffers are
 * 16-B aligned) stopped counting after the chunk holding `end`, so `capacity` counts
 * expandable candidates up to that chunk only (a lower bound; exact when the flag is clear,
 * e.g. on overflow or on the two-pass path). */
#define CODEC_PEE_PARTIAL 1
/* meta.status values: 0 ok, 1 payload exceeds capacity (truncated, still reversible),
 * CODEC_PEE_ELOOKBACK: an IN-PLACE single-pass embed's cursor look-back gave up waiting for
 * a predecessor chunk (bounded spin instead of a GPU hang; the slice's pixels are not a
 * valid stego -- the Python layer raises).  Sticky: nothing lowers it within the call.
 * Out of place a look-back that waits too long computes the missing predecessor counts
 * from the (read-only) cover itself, so the result stays exact and this never appears. */
#define CODEC_PEE_ELOOKBACK 2

/* Zero-initialise the workspace once before its first use (the diagnostic counters live
 * in it; everything else is cleared by the calls themselves).  Small out-of-place batches
 * (B <= 7) keep call-to-call state in it (status words and finished flags by call parity,
 * each carrying the call's epoch tag; the library counts the epochs per workspace).  A
 * workspace serves one call at a time: calls that share it must be ordered (one stream, or
 * synchronised); calls in flight together on different streams need separate workspaces.
 * Recovery rules:
 *   - shape change: the library remembers per (device, workspace pointer) the shape of the
 *     last call; a call of another (B, H, W, bytes) zeroes the workspace first (one extra
 *     launch; the diagnostic counters are kept, or zeroed too when the new shape places
 *     them elsewhere), so one workspace sized for the largest batch may serve smaller
 *     batches in turn;
 *   - graphs: a call made under stream capture takes the zeroing path, and the library
 *     remembers that shape as captured on the workspace.  Replays run without the host, so
 *     from then on self-cleaning calls of any OTHER shape on that workspace take the zeroing
 *     path as well (a replay may have written the captured shape's words where their finished
 *     flags lie); calls of the captured shape keep the fast path.  A fresh workspace per
 *     captured graph avoids the extra launch;
 *   - desynchronised counters (a call that never completed): a chunk reads only status words
 *     carrying its own epoch tag, so a stale word counts as "not published", the bounded
 *     wait ends in the pixel-count fallback and the results stay exact (slower;
 *     codec_pee_diag_offset counts the fallbacks).  codec_pee_reset restores the fast path;
 *   - the library keys this state by (device, pointer) and treats an unknown pointer as a
 *     fresh workspace (zeroed on its first self-cleaning call); a workspace allocated at an
 *     address an earlier one used inherits that entry, so zero-initialise it or call
 *     codec_pee_reset once (PeeCodec does so at construction);
 *   - after any failed call (non-zero return, ELOOKBACK status, a raised exception in the
 *     host layer) call codec_pee_reset before reusing the workspace: PeeCodec does so. */
size_t codec_pee_workspace_bytes(const codec_pee_params* P);
/* Re-zero the whole workspace (diagnostic counters included) on `stream` and record P's
 * shape as its owner.  No reference counterpart (workspace management only). */
int codec_pee_reset(const codec_pee_params* P, void* workspace, size_t workspace_bytes, void* stream);
/* Byte offset in the workspace of a uint32 flag that codec_pee_extract's IN-PLACE single
 * pass sets (non-zero) when a chunk's cursor look-back gave up (the recovered payload of
 * that call is not valid); cleared at the start of every codec_pee_extract.  0 on bad
 * parameters. */
size_t codec_pee_extract_flag_offset(const codec_pee_params* P);
/* Byte offset in the workspace of 4 cumulative uint32 counters (since the workspace was
 * zeroed): [0] embed / [1] extract chunks whose look-back timed out and recovered by
 * counting the missing predecessors from pixels (exact results), [2] embed / [3] extract
 * in-place chunks whose look-back timed out unrecovered.  0 on bad parameters. */
size_t codec_pee_diag_offset(const codec_pee_params* P);
/* Diagnostics: phase stamps of the last k_pee_embed_res launch run with the env knob
 * CODEC_PEE_RES_TRACE=1 (wall_clock64 at entry / end of the read phase / T chosen / ranks
 * known / end of the embed phase, 5 per workgroup, first 1024 workgroups); returns the count
 * copied or -1. */
int codec_debug_res_trace(unsigned long long* out, int n);
/* cover -> stego (full copy + expansion/shifting of candidates 0..end), lm, meta.
 * lengths[B] (device int32) = payload bits per slice.
 * stego == cover is allowed (in place): only the items up to `end` are read and
 * written, everything after `end` is left untouched.
 * Payload longer than the capacity: status 1, the first `capacity` bits are embedded,
 * end = nc - 1 (every candidate processed) and the slice stays exactly reversible. */
int codec_pee_embed(const codec_pee_params* P, const void* cover, void* stego, const uint64_t* payload,
                    const int32_t* lengths, codec_pee_meta* meta, uint64_t* lm, void* workspace,
                    size_t workspace_bytes, void* stream);
/* codec_pee_embed with a per-slice threshold: T_per_slice[B] (device int32, >= 1) replaces
 * P->T for slice b (meta.T records it; extract reads it from meta).  NULL = P->T for all.
 * Pair with codec_pee_capacity's t_out for capacity control. */
int codec_pee_embed_ts(const codec_pee_params* P, const void* cover, void* stego, const uint64_t* payload,
                       const int32_t* lengths, const int32_t* T_per_slice, codec_pee_meta* meta, uint64_t* lm,
                       void* workspace, size_t workspace_bytes, void* stream);
/* Capacity control (one read-only pass over cover; P->T is ignored, 1 <= tmax <= 64):
 * caps[B][tmax] = exact capacity of slice b at T = 1..tmax (expandable candidates whose
 * expansion stays in [0, maxval]), t_out[B] = the smallest T <= tmax whose capacity holds
 * lengths[b] bits (tmax if none does: the embed then truncates, status 1).  caps or t_out
 * may be NULL (t_out needs lengths).  Uses the PEE workspace, which must have been zeroed
 * once (its error bins are cleared at the end of every call, not at the start). */
int codec_pee_capacity(const codec_pee_params* P, const void* cover, int32_t tmax, const int32_t* lengths,
                       int32_t* caps, int32_t* t_out, void* workspace, size_t workspace_bytes, void* stream);
/* Capacity-controlled embed in one call: t_out[B] (device int32, required) receives the
 * per-slice T chosen by codec_pee_capacity's rule (1 <= tmax <= 64), and the slices are
 * embedded with it (meta.T records it) -- results identical to codec_pee_capacity(t_out)
 * followed by codec_pee_embed_ts(t_out).  Where the embed runs slice-serial (chip-filling
 * batches of small slices, or in place; uint16, tmax <= 16) the capacity pass is fused into
 * the embed launch: each slice's workgroup counts its slice, then embeds it, re-reading the
 * slice from the Infinity Cache. */
int codec_pee_embed_auto(const codec_pee_params* P, const void* cover, void* stego, const uint64_t* payload,
                         const int32_t* lengths, int32_t tmax, int32_t* t_out, codec_pee_meta* meta, uint64_t* lm,
                         void* workspace, size_t workspace_bytes, void* stream);
/* stego -> exact payload bits + restored cover.  cover_out == stego is allowed (in
 * place: only the items up to `end` are read and written). */
int codec_pee_extract(const codec_pee_params* P, const void* stego, const codec_pee_meta* meta,
                      const uint64_t* lm, void* cover_out, uint64_t* payload_out, void* workspace,
                      size_t workspace_bytes, void* stream);

/* ---- MED-PEE scheme 2: four sublattice passes (oracle/pee_cpu.py "Scheme 2"; the version-16
 * container's scheme byte 2).  Pass p (0..3) runs the scheme above on lattice p -- (odd, odd),
 * (even, even), (odd, even), (even, odd) as (row, column) parities, pixels with y >= 1 and
 * x >= 1, candidate (i, j) at (y0 + 2i, x0 + 2j) with y0 / x0 = 1 for an odd parity, 2 for an
 * even one -- on the RUNNING image, taking the next min(remaining, capacity_p) payload bits
 * of each slice: about four times scheme 1's capacity at one T.  Decoding runs the passes in
 * reverse.  metas: [4][B] codec_pee_meta (pass-major), written by the embed passes in
 * order and read by later passes (pass p's payload bits start at meta[0][b].L + ... +
 * meta[p-1][b].L); a pass with no bits left for a slice leaves it untouched (L 0, end -1,
 * capacity -1).  meta.L is the number of bits the pass embedded; meta.status 1 = the pass
 * filled up (every candidate processed); meta.reserved[0] = the lattice.  lm: this pass's
 * [B][lm_words] location map.  The PEE workspace (codec_pee_workspace_bytes) is shared with
 * scheme 1.  Passes are ordered calls on one stream. */
/* embed pass `pass`: stego = cover (copied when they differ), then the pass in place on
 * stego.  Pass 0 with cover != stego, passes 1..3 with cover == stego.  Pass 0 is scheme 1 on
 * its lattice and runs through codec_pee_embed_ts (its record's L made the embedded count;
 * an in-place pass 0 can report CODEC_PEE_ELOOKBACK like codec_pee_embed). */
int codec_pee_multi_embed_pass(const codec_pee_params* P, int32_t pass, const void* cover, void* stego,
                               const uint64_t* payload, const int32_t* lengths, codec_pee_meta* metas,
                               uint64_t* lm, void* workspace, size_t workspace_bytes, void* stream);
/* extract pass `pass` (call 3, 2, 1, 0): cover_out = stego (copied when they differ), then
 * the pass restores its lattice in place and ORs its bits into payload_out (zero it before
 * the first pass).  For pass 0 a caller may use codec_pee_extract (in place, with the pass-0
 * records and map) into a separate payload buffer and OR it in (scheme 1's kernels). */
int codec_pee_multi_extract_pass(const codec_pee_params* P, int32_t pass, const void* stego,
                                 const codec_pee_meta* metas, const uint64_t* lm, void* cover_out,
                                 uint64_t* payload_out, void* workspace, size_t workspace_bytes, void* stream);
/* Scheme 2, all four passes in one call each way (what PeeCodec(scheme=2) calls).  lm is the
 * [4][B][lm_words] maps of the four passes (pass-major), metas [4][B].  The embed runs passes
 * 0..3 (stego = cover first when they differ); the extract runs passes 3..0 (cover_out = stego
 * first when they differ) and writes payload_out [B][payload_words] whole (bits of every pass,
 * zero past them).  Results equal the per-pass calls above.  Where a chip-filling batch gives
 * every CU a slice (B >= the CU count, the last round >= 85 % full, H * W <= 2^20) a slice-
 * serial kernel takes each slice's passes in one launch (the embed's pass 0 through scheme 1's
 * copy-fused kernels first); a pass then stops counting at its `end` chunk and its capacity
 * carries CODEC_PEE_PARTIAL as scheme 1's single pass does.  Otherwise the per-pass tile
 * launches run.  No reference counterpart (the reference has no PEE code; oracle/pee_cpu.py
 * pee_embed_multi / pee_extract_multi is the specification). */
int codec_pee_multi_embed(const codec_pee_params* P, const void* cover, void* stego, const uint64_t* payload,
                          const int32_t* lengths, codec_pee_meta* metas, uint64_t* lm, void* workspace,
                          size_t workspace_bytes, void* stream);
int codec_pee_multi_extract(const codec_pee_params* P, const void* stego, const codec_pee_meta* metas,
                            const uint64_t* lm, void* cover_out, uint64_t* payload_out, void* workspace,
                            size_t workspace_bytes, void* stream);

/* ---- exchange records of the MED-PEE side information (north star: "an RCCL all-gather of
 * per-slice location maps"; no reference counterpart -- the reference is
 * single-process).  Record b = CODEC_PEE_RECORD_HDR_WORDS uint64 words holding slice b's
 * codec_pee_meta, then `width` words of location map:
 *   sparse (meta.lm_count <= 2 * width): the candidate indices of the map's set bits,
 *          ascending, as uint32 (two per word), unused slots zero;
 *   dense  (otherwise): map words 0 .. width-1 with every bit past `end` zero.
 * Slice b's map travels exactly when width >= min(ceil(lm_count / 2), ceil((end + 1) / 64)).
 * meta/lm: codec_pee_embed outputs ([B], [B][lm_words]); records: [B][HDR + width]. */
#define CODEC_PEE_RECORD_HDR_WORDS 8
/* set in a packed record's meta.flags when the map held fewer set bits in [0, end] than
 * meta.lm_count said (the record's lm_count is then the number found and travels sparse) */
#define CODEC_PEE_RECORD_RECOUNTED 2
int codec_pee_pack_records(int32_t B, int32_t lm_words, const codec_pee_meta* meta, const uint64_t* lm,
                           int32_t width, uint64_t* records, void* stream);
/* Inverse for n gathered records: meta_out[n] (may be NULL) and lm_out[n][lm_cols] (may be
 * NULL) = each slice's location map, dense, zero past `end` and truncated to lm_cols words. */
int codec_pee_unpack_records(int32_t n, int32_t width, const uint64_t* records, int32_t lm_cols,
                             codec_pee_meta* meta_out, uint64_t* lm_out, void* stream);

/* ---- stego quality (replaces the metric arithmetic of src/mse.py: AnalisadorMSE.
 * calcular_mse :74-117, calcular_psnr :119-133, calcular_ssim_simples :135-177 and the
 * difference statistics of analisar_par_imagens :201-207).  One read-only pass over two
 * [B][H][W] images of `bytes` (1 or 2) per pixel writes per slice 10 exact uint64
 * moments out[B][10] = {sum a, sum b, sum a^2, sum b^2, sum a*b, sum |a-b|, max |a-b|,
 * count(a != b), max a, max b}; the metrics are closed forms of them
 * (codec_tcc_amd/quality.py evaluates them in exact rational arithmetic). */
#define CODEC_QUALITY_WORDS 10
int codec_quality_moments(int32_t B, int32_t H, int32_t W, int32_t bytes, const void* a, const void* b,
                          uint64_t* out, void* stream);

/* ---- measurement hooks (bench.py): while a profile window is open, every launcher
 * records a hipEvent pair around each kernel it launches, tagged with a CODEC_K_* id.
 * Events are created/destroyed here, outside any launch function. */
#define CODEC_K_SCAN_FAST 1
#define CODEC_K_SCAN_GENERIC 2
#define CODEC_K_BLOCK_EXACT 3
#define CODEC_K_DECIDE 4
#define CODEC_K_EMBED 5
#define CODEC_K_RESTORE 6
#define CODEC_K_GATHER 7
#define CODEC_K_OTHER 8
#define CODEC_K_PEE_SCAN 9
#define CODEC_K_PEE_LOCATE 10
#define CODEC_K_PEE_EMBED 11
#define CODEC_K_PEE_COPY 12
#define CODEC_K_PEE_DCOUNT 13
#define CODEC_K_PEE_RECOVER 14
#define CODEC_K_PEE_EMBED1 15
#define CODEC_K_PEE_EXTRACT1 16
#define CODEC_K_SCAN_READ 17
#define CODEC_K_UNXOR 18
#define CODEC_K_SCAN_ROWS 19
#define CODEC_K_SCAN_ROWS_READ 20
#define CODEC_K_QUALITY 21
#define CODEC_K_DECIDE_EMBED 22
#define CODEC_K_PEE_CAPACITY 23
#define CODEC_K_PEE_EMBED_SS 24
#define CODEC_K_PEE_EXTRACT_SS 25
#define CODEC_K_PEE_EMBED_SS_AUTO 26
#define CODEC_K_PEE_EMBED_RES 27   /* resident auto embed: slice read once, kept on the CU */
#define CODEC_K_SCAN_DECIDE 28     /* fused scan + decide + embed (one workgroup per slice)  */
#define CODEC_K_PEE_LAT_COUNT 29   /* scheme 2: one pass's tile counts + per-slice locate      */
#define CODEC_K_PEE_LAT_EMBED 30   /* scheme 2: one pass's in-place embed                      */
#define CODEC_K_PEE_LAT_DCOUNT 31  /* scheme 2: one pass's decodable-bit counts + offsets      */
#define CODEC_K_PEE_LAT_RECOVER 32 /* scheme 2: one pass's in-place recovery                   */
#define CODEC_K_PEE_LAT_SS_EMBED 33   /* scheme 2 slice-serial: copy + embed passes, one launch  */
#define CODEC_K_PEE_LAT_SS_EXTRACT 34 /* scheme 2 slice-serial: copy + every extract pass         */
int codec_profile_begin(int32_t capacity);
/* after the stream has been synchronised: fills ms[i], tag[i] for the recorded pairs and
 * returns their count (closes the window and frees the events). */
int codec_profile_end(float* ms, int32_t* tag, int32_t capacity);

#ifdef __cplusplus
}
#endif
#endif /* CODEC_TCC_H */
