// amx_internal.hpp -- device-visible plan structures shared by amx_kernels.hip
// (CDNA4 kernels) and amx_plan.cpp (host plan construction + C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define AMX_MAX_EQ_DIM 20
#define AMX_XO_DIM 8      // crossover: 2 low-pass + 2 high-pass SOS sections
#define AMX_KW_DIM 4      // K-weighting 4th-order DF-II state (v1..v4)
#define AMX_BLOCK 256
#define AMX_HIST_BINS 1000
#define AMX_TF_FRAMES 16  // LDS tile frames (AMX_TF in amx_dev.hpp)
#ifndef AMX_SCAN_S
#define AMX_SCAN_S 16     // segments per scan block
#endif
#define AMX_SCAN_PW 6     // window powers staged in LDS by the down sweep (more: read from memory)
#define AMX_CTL_FAST 1    // k_decide control word: limiter provably idle
#define AMX_STATS 16      // doubles per track written by k_decide
#define AMX_ENV_MAX_ROUNDS 16  // envelope fix-up flag words (k_env0 clears them)
#define AMX_ENV_NCTR 4         // fix-up diagnostic counters per round (after the flags; k_envchain)
#define AMX_ENV_BACT (AMX_ENV_MAX_ROUNDS * (1 + AMX_ENV_NCTR))  // band-activity words after the counters
#define AMX_ENV_LIST (AMX_ENV_BACT + 4)  // re-run list length, chain-head list length, k_envseq's flag
#define AMX_EQC 64        // compact EQ coefficient block (see ChainDev::eqc)
#define AMX_MEAS_RATE 192000  // loudnorm pass 1 measures at 192 kHz (af_loudnorm dynamic mode)
#ifndef AMX_PCM_U8        // input PCM formats (include/amx.h amx_pcm_to_s16)
#define AMX_PCM_U8 0
#define AMX_PCM_S16 1
#define AMX_PCM_S24 2
#define AMX_PCM_S32 3
#define AMX_PCM_F32 4
#define AMX_PCM_F64 5
#define AMX_PCM_S8 6
#define AMX_PCM_S16BE 7
#define AMX_PCM_S24BE 8
#define AMX_PCM_S32BE 9
#define AMX_PCM_F32BE 10
#define AMX_PCM_F64BE 11
#endif

// One EQ stage of _apply_eq_to_channel (audio_mastering_engine.py:277-282).
struct EqStageDev {
    int32_t kind;    // 0 skipped, 1 shelf (lfilter ba, :283-289), 2 peak (4 SOS, :290-298)
    int32_t neg;     // shelf with gain_db < 0 (:289)
    double g;        // 10**(gain_db/20)
    double gm1;      // g - 1
    float gf;        // float32(g): the float32 product of :289 on a float32 input
    float pad_;
    double c[24];    // shelf: b0 b1 b2 a0 a1 a2 ; peak: 4 x [b0 b1 b2 a0 a1 a2]
};

struct ChainDev {
    int32_t fs, chin;
    int32_t in_s16, pad0_;
    int32_t analog_on, has_lut;
    int32_t eq_mask, eq_dim;
    int32_t width_on, mb_on;
    float width, drive;
    double an_lo[6];
    double an_glo1;   // analog low shelf g - 1
    double an_hi[6];
    double an_ghi1;
    EqStageDev st[4];
    double xlo[12], xhi[12];
    // compressor (pydub compress_dynamic_range, :306-308)
    int32_t look;          // int(5 ms * fs)
    int32_t rthr[3];       // smallest integer rms with rms > thresh_rms
    int32_t rq[3];         // first table index r with m(r) != 0 (32769: none); r < rq is quiet
    int32_t pad_rq_;
    double kw1[6], kw2[6]; // K-weighting as two DF-II-T biquads (libebur128 pb/pa, rb/ra)
    // Active EQ stages packed in order for register-resident use (amx_dev.hpp eq_chain):
    //   shelf: b0 b1 b2 a1 a2 gx     (gx = g-1, or the negative-gain factor g / f32(g))
    //   peak : 4 x [b0 b1 b2 a1 a2] gm1
    double eqc[AMX_EQC];
    // envelope divisions inc = m / A, dec = m / R (pydub frame counts): env_rcp = 1
    // when the reciprocal-multiply with one FMA correction was checked on the host to
    // equal the IEEE quotient for every table value m (amx_dyn.hip env_div)
    double env_A, env_R, env_rA, env_rR;
    int32_t env_rcp;
    // k_env0's warm-up start guess: 1 = m of the warm-up's first frame, 0 = att = 0
    // 
    int32_t env_guess;
    // envelope segment tables by active-band count (amx_dyn.hip): table t (1..3) cuts
    // the chunks into segments of Le frames so that t bands' segments fill the CUs as
    // one resident wave set; k_rms flags the bands with a frame over the threshold and
    // the envelope kernels take the table of that count.  Offsets index the plan's
    // concatenated segment array and per-chunk (first, count) arrays; the per-band
    // segment arrays (s, e, act, prev) have stride es_ld = the largest n_es
    int32_t es_ld;
    struct { int32_t es_off, n_es, ch_off, Le; } etab[4];
    // exp10 constants of the gain (amx_dyn.hip exp10_gain): read through the plan so
    // they are scalar operands of the FMAs (a 64-bit literal is not encodable)
    double exc[16];
};

// A ~30 s chunk (ffmpeg segment, :178).  loc_off indexes chunk-local scratch.
struct ChunkDev {
    int64_t in_off;    // first input frame in d_in
    int64_t loc_off;   // offset in per-frame scratch arrays (sum of previous chunk lengths)
    int64_t out_off;   // offset in d_out (frames)
    int64_t n;         // input frames
    int64_t out_n;     // output frames (n, or pydub overlay ms-rounded length when multiband)
    int32_t seg0, nseg;
    int32_t track, pad_;
};

// IIR / envelope segment: `len` frames from chunk-local frame `pos`.
struct SegDev {
    int64_t pos;
    int32_t chunk;
    int32_t len;
    int32_t first;     // global index of the first segment of the same chunk
    int32_t last;      // 1 if last segment of its chunk
};

// K-weighting segment over a track span of d_out.
struct KwSegDev {
    int64_t out_pos;     // frame in d_out
    int64_t tframe;      // frame in the whole-track timeline
    int32_t track;
    int32_t len;
    int32_t first;       // global index of the span's first segment (the scan stream)
    int32_t last;        // 1 if last segment of its span
};

// A block of up to AMX_SCAN_S consecutive segments of one stream (amx_scan.hip).
struct ScanBlk {
    int32_t seg0, nseg;
    int32_t first;       // index of the stream's first block
    int32_t last;        // 1 if the stream's last block
    int32_t stream, pad_;
};

struct SpanDev {
    int64_t out_off, out_n, tframe0, ttotal;   // chain-output frames (d_out) of the span
    int32_t kseg0, nkseg;
    // the loudness measurement's stream (192 kHz when resampled, else == the chain's):
    // first frame of the span in the whole track, frames of the span, of the track
    int64_t m_tframe0, m_n, m_total;
    int32_t edge_lo, edge_hi;   // resampler window past the span start / end reads the
                                // neighbour rank's frames (edge buffer), else mirrors
};

// ---------------------------------------------------------------- launchers
namespace amx {
// pass 1 for float32 stereo input with the analog stage: k_analog_h + k_gemv16 (the odd
// tanh table's half in LDS; default), or k_front1s with the full table in global memory
// (a table that is not odd; AMX_F1 = 2 forces it, for tests)
#define AMX_F1_SPLIT 0
#define AMX_F1_FULL 2
struct Launch {
    const ChainDev *cd;
    const ChunkDev *chunks;
    const SegDev *segs;
    int32_t n_chunks, n_seg, L;
    hipStream_t stream;
    const float *lut_half = nullptr;   // odd tanh table's half (k_analog_h), NULL: the full table
    int f1_mode = AMX_F1_SPLIT;        // float32 stereo + analog: which pass-1 form (amx_chain.hip)
    int64_t max_chunk_n = 0;           // frames of the longest chunk (elementwise grids)
    int64_t an_blocks = 0;             // k_analog_h's 4096-frame blocks over all chunks
    int an_vec = 0;                    // every chunk: even in_off and >= 4 frames (k_analog_h<true>)
};
struct ScanPlan {
    int D, n_blk, K;
    const ScanBlk *blks;
    const double *M;     // A^L, D x D row-major
    const double *Mbk;   // (A^{L S})^k, k = 1 .. K-1
};
hipError_t launch_front1(const Launch &l, int D, int win, bool analog, const float *in,
                         const float *lut, int16_t *a16, const double *G, double *e, bool sc = false);
// tailP / tail (the K filter, D = 4): the down sweep also writes each stream's end state
// P_t s_last + e_last (k_kw_tail's product) from its last block
hipError_t launch_scan(const ScanPlan &p, const double *e, double *s, const double *carry,
                       double *eb, hipStream_t st, bool up = true, const double *tailP = nullptr,
                       double *tail = nullptr);
hipError_t launch_front2(const Launch &l, int mask, const int16_t *a16, const double *s_eq,
                         int16_t *dst, int to_out, const double *Gx, double *e_x,
                         const double *Gkw, double *e_kw, uint32_t *pk, bool sc = false,
                         const float *slut = nullptr);
hipError_t launch_xover2(const Launch &l, const int16_t *p16, const double *s_x,
                         int16_t *bands, int64_t nloc, int *bact);
struct DynLaunch {
    const ChainDev *cd;
    const ChunkDev *chunks;
    int n_chunks;
    const SegDev *es;            // envelope segments: the tables of ChainDev::etab, concatenated
    int n_es;                    // the largest table's segment count (= ChainDev::es_ld)
    const int *eseg0, *neseg;    // per chunk: first envelope segment, count
    int64_t nloc, max_chunk_n;
    int look, warm, Le, rcp;
    const double *tabs;
    hipStream_t st;
    int env_wg, env_pin;         // k_env0: waves per workgroup, one workgroup per CU
};
hipError_t launch_rms(const DynLaunch &d, const int16_t *bands, uint16_t *m, int *bact);
// C > 2 channels (round 6): the bands of a stream sub-plan (schunks, snloc), r / the
// checkpoints / the output on the real frames of the plan in d
hipError_t launch_mc_rms(const DynLaunch &d, const ChunkDev *schunks, const int16_t *bands, int64_t snloc,
                         int C, uint16_t *m, int *bact);
hipError_t launch_mc_gain_overlay(const DynLaunch &d, const ChunkDev *schunks, const uint16_t *m,
                                  const double *ck, const int16_t *bands, int64_t snloc, int C,
                                  int64_t max_chunk_out, const int64_t *n1tab, const int *bact, int16_t *out);
hipError_t launch_mc_pack(const void *in, int64_t samples, int in_s16, uint32_t *pairs, hipStream_t st);
hipError_t launch_mc_unpack(const uint32_t *pairs, int64_t samples, int16_t *out, hipStream_t st);
hipError_t launch_mc_split_pairs(const int16_t *y, int64_t frames, int C, int16_t *pairs, hipStream_t st);
hipError_t launch_mc_loudness_combine(const double *hops, int64_t max_hops, const double *peak, int C,
                                      double *hops1, double *peak1, hipStream_t st);
hipError_t launch_mc_peak_pick(const int16_t *y, int64_t frames, int C, const double *gain, int16_t *syn,
                               hipStream_t st);
hipError_t launch_mc_limiter_out(const int16_t *y, int64_t frames, int C, int halo_frames, const double *gains,
                                 const int32_t *ctl, const double *att, double level_in, double level,
                                 double level_out, double limit, int16_t *out, hipStream_t st);
// input decode: PCM of any supported format -> stereo s16 frames (amx_io.hip)
hipError_t launch_zero(void *p, size_t bytes, hipStream_t st);   // a kernel, never a memset node
hipError_t launch_pcm_to_s16(const void *raw, int64_t frames, int channels, int fmt, int16_t *out,
                             hipStream_t st);
hipError_t launch_env(const DynLaunch &d, const uint16_t *m, double *ck, double *sv, double *ev,
                      int *act, int *list, int *hmark, int *prev, int *list0, int *flags, int rounds,
                      int part);
hipError_t launch_envseq(const DynLaunch &d, const uint16_t *m, double *ck, double *sv, double *ev,
                         const int *act, const int *flags, int rounds);
hipError_t launch_gain_overlay(const DynLaunch &d, const uint16_t *m, const double *ck,
                               const int16_t *bands, int16_t *out, int64_t max_chunk_out,
                               const int64_t *n1tab, const int *act, const int *bact);
// loudness
// gate (amx_plan_set_gate): the kernel returns at once unless the word says dynamic
hipError_t launch_kw1(const ChainDev *cd, const KwSegDev *ks, int n_kseg, int L,
                      const int16_t *x, const double *G, double *e, uint32_t *pk,
                      const int32_t *gate, hipStream_t st);
hipError_t launch_kw2(const ChainDev *cd, const KwSegDev *ks, int n_kseg, int L, int hop,
                      const int16_t *x, const double *s, double *parts, int64_t *part_hop,
                      int aligned, const int32_t *gate, hipStream_t st);
hipError_t launch_hops(const SpanDev *spans, int n_tracks, const KwSegDev *ks, int L, int hop,
                       const double *parts, const int64_t *part_hop, double *hops,
                       int64_t max_hops, hipStream_t st);
hipError_t launch_hist(const SpanDev *spans, int n_tracks, int hop, const double *hops,
                       int64_t max_hops, const double *bounds, unsigned long long *hist,
                       unsigned long long *st_hist, hipStream_t st);
// loudness at 192 kHz (amx_loud192.hip): the resampled stream is recomputed from d_out
#define AMX_UP_EDGE 80     // frames of the neighbour rank's output the resampler window needs
                           // (16 for the 32-tap upsampler; up to 67 for 768 kHz's 132 taps)
#define AMX_SWR_MAX_ALLOC 144   // the widest resampler row (filter_alloc) restated
#define AMX_UP_BLOCK 64
// k_up_poly's template form as one code (launch switch, plan)
#define AMX_UP_POLY(cmin, cmax, tb) ((cmin) * 256 + (cmax) * 16 + (tb))
int up_poly_form(int cmin, int cmax, int tb);   // the code if that form is built, else 0
struct UpArgs {
    const ChainDev *cd;
    const KwSegDev *ks;
    int n_kseg;
    const SpanDev *spans;
    int Lin, Lout;            // input frames / 192 kHz outputs per K segment
    int static_l;             // L when M == 1 (unrolled kernels), else 0 (tables)
    int poly;                 // k_up_poly's form (AMX_UP_POLY), else 0
    const int32_t *fcnt;      // k_up_poly: per segment frame, the outputs it is the base of
    const float *bankn;       // k_up_poly: [Lout][32] the bank rows in output order
    int hop;
    const int32_t *obase, *oph;   // per output n < Lout: input frame (segment-relative), phase
    const float *owt;             // per output: interpolation weight (lin)
    int lin;                      // libswresample's linear kernel: rows oph, oph + 1 (1024 phases)
    const int32_t *slow;          // segments k_up_slow takes (NULL: all, when static_l == 0)
    int64_t n_slow;
    const float *bank;            // [pc + 1][alloc] float32 polyphase bank (row pc = row 0 one tap on)
    int taps, alloc;              // filter_length, filter_alloc: 32, 32 but for downsampling rates
                                  // (then every segment goes through k_up_wide)
    const uint32_t *x, *edge;     // d_out (stereo s16 dwords); edge [tracks][2][AMX_UP_EDGE]
    const double *G;              // rows C A^n, n < Lout (the K filter's free response)
    const double *qh, *qt;        // Gram matrices of those rows: head sums [Lout+1][16], tail sums
    double *eterms;               // [seg][ch][10]: per hop piece sum yz^2, sum yz (C A^n)^T
    double *e;
    const double *s;              // segment start states (after the scan)
    double *parts;
    int64_t *part_hop;
    uint32_t *pk;                 // [seg][4]: 192 kHz |u| max L, R (float bits), native |x| L, R
};
// af_loudnorm's 192 kHz modes on one whole track (amx_loudnorm.hip)
struct LnArgs {
    int64_t n192;                 // 192 kHz frames
    float *u;                     // [n192][2] the resampled stream (scratch)
    double *ring;                 // limiter ring [40320][2] + 64 (scratch)
    int16_t *y;                   // [n192][2] output
    double *summary;              // [2]: 1 = the < 3 s linear fallback ran (then [1] = its offset)
    const double *hops;           // [>= n192 / 19200][2] pass-1 hop energies of this stream
    const double *peak;           // [2] pass-1 192 kHz sample peak per channel
    const double *energies, *bounds;
    double target_i, target_lra, target_tp;   // target_tp linear (the ceiling)
    double measured_i, measured_thresh, offset;   // offset linear
    double weights[21];           // init_gaussian_filter
    double kb[5], ka[5];          // libebur128 K filter at 192 kHz (direct form)
    // set when the parallel form (LpArgs) runs first: this kernel then only runs the
    // tracks it hands over (lp_ctl[0] != 0) with the options it resolved (lp_dctl)
    int *lp_ctl;
    const double *lp_dctl;
    // a quiet start (above_threshold 0) runs here only until the output's short-term
    // loudness lifts it: at the next segment start the state is handed to the parallel
    // form (lp_recG[k] holds it, lp_D the deltas written so far); INNER segment k >= 1
    // starts at frame 1 + k lp_Fs, k <= lp_J
    double *lp_D, *lp_recG;
    int lp_Fs, lp_J;
    // (chunk-sharded quiet start, amx_ln_shard.part 3) the first INNER frame this kernel may
    // not run: rank 0 holds the frames before it; a track still quiet there is left to
    // the replicated form (lp_ctl[0] stays 1).  INT_MAX otherwise.
    int lp_tstop;
};
// af_loudnorm dynamic mode in parallel form (amx_loudnorm.hip):
// per-frame statistics and gains from pass 1's hop energies, then the true-peak
// limiter as warmed-up segments of 100 ms frames with an in-order check and repair.
#define AMX_LN_RING 40320          // frame_size(192000, 210): the limiter ring, frames
#define AMX_LN_WIN 2048            // ring frames compared at a segment boundary
#define AMX_LN_REC (16 + 2 * AMX_LN_WIN)   // doubles of one boundary state record
#ifndef AMX_LP_NT
#define AMX_LP_NT 256    // lanes of a k_lp_seg / k_lp_walk workgroup (amx_loudnorm.hip)
#endif
struct LpArgs {
    int64_t n;                    // 192 kHz frames
    int64_t S0;                   // first output frame of the FINAL (flush) frame
    int T, nb_last;               // INNER frames, frames of the last one
    int Fs, Wf;                   // frames per segment, warm-up frames
    int J, M, K, P;               // INNER segments after segment 0, FINAL segments, all, waves
    const float *u;               // [n][2] the resampled stream
    const double *hops;           // [>= n / 19200 + 1][2] pass-1 hop energies (r128_in)
    const double *energies, *bounds;
    double target_i, target_lra, ceiling, measured_i, measured_thresh, offset;  // host values
    const double *measured_src;   // non-NULL: measured I / thresh from this k_decide row ([4], [7])
    const double *offset_src;     // non-NULL: offset = "%.2f"(target_i - offset_src[0]) dB
    const int32_t *gate;          // non-NULL: run only if this k_decide control word says dynamic
    double weights[21];
    double *v;                    // [T] AGC value of each INNER frame (when not held)
    int *hold;                    // [T] 1: the frame keeps the previous delta
    double *D;                    // [T] delta written by each INNER frame
    double *G;                    // [T + 1] Gaussian-smoothed gain of each INNER frame, FINAL's
    double *ramp;                 // [19200] i / 19200.0
    double *recG, *recE;          // [K][AMX_LN_REC] guessed start / end states per segment
    double *wrec;                 // [2][AMX_LN_REC] walker-made end states
    int *cnt, *match;             // [K + 1] boundary arrivals, start guess == previous end
    double *rings;                // [P][AMX_LN_RING][2] per-wave limiter rings
    double *wring;                // [AMX_LN_RING][2] the walker's ring
    int *ctl;                     // [16] 0: 0 parallel, 1 frame by frame (k_ln_dyn), 2 handed over,
                                  // 3 gated off, 4 quiet start run by k_ln_dyn up to segment
                                  // ctl[4], parallel from there; 1 re-runs, 2 FINAL re-run,
                                  // 3 above_threshold at FIRST, 5 frame of the hand-over
    double *dctl;                 // [8] 0 d0, 1 offset (linear), 2 measured_i, 3 measured_thresh,
                                  // 4 offset (dB)
    int16_t *y;                   // [n][2] output
    double *summary;              // [16]
    // a chunk-sharded track's share (amx_loudnorm_192k_shard): k_lp_seg runs the segments
    // [kb, ke), k_lp_walk walks their boundaries from rec_in (NULL: from the track start)
    // and leaves the true state at ke in rec_out (NULL: none); whole track: 0, K, NULL, NULL
    int kb, ke;
    const double *rec_in;
    double *rec_out;
    // [n / 64 + 2] the largest |unlimited value| per 64 positions (k_lp_fill); non-NULL:
    // k_lp_fill writes every position's unlimited output first, lp_detect skips blocks
    // below the ceiling and k_lp_seg emits only the multiplied slots
    double *bm;
    // [n / 64 + 2] the same bound for FINAL's frames: the largest |u G_T offset| per 64
    // positions from S0 (FINAL refills the whole ring with those values); NULL with bm
    double *bmF;
};
// the 192 kHz resampler's geometry (amx_plan.cpp swr_*): output j sits at phase
// position j dst / src (units of 1 / pc input frame); lin: interpolate rows ph, ph + 1
struct SwrDev {
    int pc, lin;
    int64_t src, dst;
    const float *bank;            // [pc + 1][alloc]
    int taps, alloc;              // filter_length, filter_alloc (32, 32 but downsampling)
};
// resample false: ln.u already holds the stream (amx_loudnorm_desc.reuse_stream)
hipError_t launch_loudnorm(const LnArgs &a, const LpArgs &p, const uint32_t *x, int64_t n_in,
                           const SwrDev &r, bool resample, hipStream_t st);
hipError_t launch_loudnorm_shard(const LnArgs &a, const LpArgs &p, const uint32_t *x, int64_t n_in,
                                 const SwrDev &r, int64_t u_lo, int64_t u_hi, int64_t y_lo, int64_t y_hi, int part,
                                 bool resample, hipStream_t st);
#define AMX_LN_GATED(g) ((g) && (((g)[0] >> 4) & 15) != 3)   // k_decide mode 3 = dynamic
hipError_t launch_up1(const UpArgs &a, hipStream_t st, hipStream_t aux, hipEvent_t fork, hipEvent_t join);
int swr_geometry(int in_rate, int out_rate, int *L, int *M);   // host (amx_plan.cpp)
int swr_phases(int in_rate, int out_rate);
int swr_incr(int in_rate, int out_rate, int64_t *src_incr, int64_t *dst_incr);
int swr_bank(int in_rate, int out_rate, float *bank);
hipError_t launch_up2(const UpArgs &a, hipStream_t st);
// finalize
// general alimiter scratch (plan-owned, amx_limiter_prepare): per segment of
// seg_frames frames the guessed start state G and the end state E (warm-up of
// warm_frames frames from rest), finished-block counters
#define AMX_LIM_SEG_DEFAULT 16384
#define AMX_LIM_MAX_BLOCKS 2048
struct LimScratch {
    double *seg_state = nullptr;   // [tracks][max_segs][2][state_doubles]
    unsigned *cnt = nullptr;       // [tracks], zero between launches
    int seg_frames = 0, warm_frames = 0, max_segs = 0, buffer_size = 0;
    int64_t warm_cap = 0;          // furthest warm-up start before a segment, frames
    const int32_t *gate = nullptr; // amx_plan_set_gate: k_final returns unless dynamic
    double *att = nullptr;         // amx_plan_set_limiter_trace: per output frame att, or NULL
};
size_t limiter_lds_bytes(int buffer_size);
#define AMX_LIM_LDS_MAX (160 * 1024)   // gfx950: one workgroup may hold a CU's whole LDS
hipError_t limiter_allow_lds(size_t bytes);   // k_final's dynamic LDS limit raised to it
hipError_t launch_final(const SpanDev *spans, int n_tracks, int64_t max_span, const int16_t *x,
                        const int16_t *halo, int halo_frames, const double *gains,
                        const int32_t *ctl, int fast, int fs, double level_in, double level,
                        double level_out, double limit, double release, int buffer_size,
                        double *state, int64_t state_doubles, int from_rest, const LimScratch &ls,
                        int16_t *y, hipStream_t st);
struct DecideArgs {
    int n_tracks, lufs_on;
    const unsigned long long *hist, *st_hist;
    const double *peak, *energies, *bounds;
    double target_i, target_tp, target_lra, level_in, limit;
    double *stats, *gains;
    int32_t *ctl;
    int32_t *host_ctl;     // amx_plan_set_publish: the words also into pinned host memory
};
hipError_t launch_decide(const DecideArgs &a, hipStream_t st);
hipError_t launch_publish(const int32_t *ctl, int32_t *host, int n, hipStream_t st);
hipError_t launch_kw_carry(const double *tails, const double *P, int n_prev, double *carry,
                           hipStream_t st);
hipError_t launch_kw_carry_rows(const double *rows, int world, int ld, const double *P, int n_prev,
                                double *carry, double *peak, hipStream_t st);
// per-track sample peak: partial maxima per block into part[track][block][2], the last
// block of a track (counter cnt[track], zero between launches) writes peak[track][2]
int peak_reduce_blocks(int64_t max_nkseg);
hipError_t launch_peak_reduce(const SpanDev *spans, int n_tracks, int64_t max_nkseg,
                              const uint32_t *pk, double *peak, unsigned int *cnt, int *part,
                              const KwSegDev *ks, int L, const int16_t *x, const double *G,
                              double *e, int kw_fix, int resamp, hipStream_t st);
hipError_t launch_kw_tail(const SpanDev *spans, int n_tracks, const double *s, const double *e,
                          const double *P, double *tail, hipStream_t st);
}  // namespace amx
