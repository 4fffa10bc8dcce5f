/*
 * amx.h -- C ABI of libamx.so, the MI355X-native mastering DSP hot path.
 *
 * Drop-in boundary for the reference's per-chunk mastering pipeline
 * (theouterlimitz/Audio-Mastering-Engine, audio_mastering_engine.py):
 *
 *   reference interface                                  | replaced by
 *   -----------------------------------------------------+-------------------------------
 *   chunk loop :185-204 (AudioSegment -> analog :192,    | amx_run_chunks()
 *     float :193, EQ :194, width :195, int16 :196,       |
 *     multiband :197) + ffmpeg concat :205-214           |
 *   normalize_loudness_on_disk_with_ffmpeg :227-246      | amx_loudness_pass1/pass2(),
 *     (ffmpeg loudnorm pass 1 measurement :229-237)      | amx_loudness_histograms()
 *   loudnorm pass 2 (linear mode) :240-242 +             | amx_finalize()
 *     final alimiter :223                                |
 *   process_audio_with_ffmpeg_pipeline :171-226          | host: amx/engine.py master_audio()
 *
 * Conventions:
 *  - every function returns AMX_OK (0) or a negative AMX_E* code; amx_last_error()
 *    returns a thread-local message for the last failure on the calling thread;
 *  - the caller owns every device pointer it passes (input, output, workspace);
 *    the plan owns only its small constant tables;
 *  - device calls are asynchronous on the given hipStream_t (passed as void*);
 *    they never allocate, copy synchronously or synchronise, so they may be
 *    captured into a hipGraph;
 *  - one plan per stream/thread; plans are not shared across threads;
 *  - no torch types cross this ABI; multi-GPU exchange (RCCL all-reduce of the
 *    loudness partials, K-filter carry all-gather) is done by the host between
 *    calls, on buffers this ABI fills and consumes.
 */
#ifndef AMX_H
#define AMX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AMX_OK 0
#define AMX_EINVAL -1     /* bad argument / settings */
#define AMX_EHIP -2       /* HIP runtime error */
#define AMX_ENOMEM -3     /* host allocation failed */
#define AMX_ERANGE -4     /* a size or filter is outside what the plan supports */

/* ABI history.  3 -> 4 (round 6): amx_loudnorm_desc gained reuse_stream (the struct
 * grew), amx_ln_shard.pad_ became `windowed`, d_edge went from [2][16][2] to [2][80][2]
 * frames per track, amx_final_desc.pad_ became `from_rest`.  A caller built against
 * an older header must be rebuilt: amx_abi_version() tells it which layout it gets. */
#define AMX_ABI_VERSION 4

#if defined(__GNUC__)
#define AMX_API __attribute__((visibility("default")))
#else
#define AMX_API
#endif

/* Filter coefficients and parameters of the chain.  The host designs them with
 * the same calls the reference makes (scipy.signal.butter at :285, :296,
 * :301-302), so the device sees the reference's exact numbers. */
typedef struct amx_chain_desc {
    int32_t sample_rate;
    int32_t channels_in;          /* 1 or 2; mono is duplicated to stereo (:190) */
    int32_t input_s16;            /* 0: d_in is float32 (quantised on device like ffmpeg's
                                     f32->s16 segment split, A.1); 1: d_in is int16 already
                                     (mono int16 is duplicated to stereo on the device) */
    int32_t measure_only;         /* 1: the plan only measures / limits a track it is given in
                                     d_out (amx_run_chunks is not called): loudness pass 1
                                     then runs its own sample pass instead of the one
                                     k_front2 fuses into the chain */
    /* analog character (:258-266), applied if analog_on */
    int32_t analog_on;
    float analog_drive;           /* float32(1 + 0.5*cf) */
    const float *tanh_lut;        /* 65536 float32: tanh(float32(s/32768)*drive) for
                                     s = -32768..32767 (numpy's float32 tanh); required
                                     when analog_on */
    double analog_lo_ba[6];       /* butter(2,120/(fs/2),'low'):  b0 b1 b2 a0 a1 a2 */
    double analog_lo_gain;        /* 10**(cf/20) */
    double analog_hi_ba[6];       /* butter(2,12000/(fs/2),'high') */
    double analog_hi_gain;        /* 10**(1.5cf/20) */
    /* 4-stage EQ (:277-282): stage order low shelf 250 Hz, peak 1 kHz, peak 4 kHz,
     * high shelf 8 kHz.  kind 0 = skipped (gain 0), 1 = shelf (ba in coef[0..5]),
     * 2 = peak (4 SOS rows [b0 b1 b2 a0 a1 a2] in coef[0..23]). */
    int32_t eq_kind[4];
    double eq_gain_db[4];
    double eq_gain[4];            /* 10**(gain_db/20) */
    double eq_coef[4][24];
    /* stereo width (:267-271) */
    int32_t width_on;
    float width;
    /* multiband (:299-309) */
    int32_t multiband_on;
    double xover_lo_sos[12];      /* butter(4,250,'lowpass',fs,sos) */
    double xover_hi_sos[12];      /* butter(4,4000,'highpass',fs,sos) */
    double comp_threshold_db[3];  /* low, mid, high */
    double comp_ratio[3];
    const double *comp_m_table[3];/* optional override of max_attenuation(rms), rms=0..32768;
                                     NULL -> the plan tabulates it with the C library's
                                     log/pow, which is what CPython's math uses (pydub) */
    /* compressor envelope parallelisation (amx_dyn.hip); results are exact for any
     * values, these only move work between the speculative and the fix-up passes */
    int32_t env_warm_frames;      /* speculative warm-up per envelope segment (rounded up to 128); <0 -> 2304 */
    int32_t env_rounds;           /* parallel fix-up rounds before the in-order walk (0..16); <0 -> 2 */
    /* (ABI 4) a chain over ONE interleaved 1-D stream: the sub-plans amx_mc_plan_create
     * builds for a file with more than two channels (audio_segment_to_float_array only
     * reshapes stereo, :252).  The stream is the L channel of a pseudo-stereo int16
     * buffer (R = 0).  stream_chain = 1: the EQ result is clipped and scaled in float64
     * when a stage ran (the 1-D branch of :273-275 keeps float64), in float32 when none
     * did; width, analog and mono input are refused.  eq_in_lut (nullable): the input
     * sample s enters the EQ as eq_in_lut[s + 32768] instead of s / 32768 (the analog
     * character of a stream: float32 tanh, then its two shelves ALONG the stream, run
     * as EQ stages 0 and 3). */
    int32_t stream_chain;
    int32_t pad_sc_;
    const float *eq_in_lut;
} amx_chain_desc;

/* One ~30 s chunk of one track (the ffmpeg segment split, :178). */
typedef struct amx_chunk {
    int32_t track;                /* track index within the plan */
    int32_t pad_;
    int64_t in_offset;            /* first input frame of the chunk in d_in */
    int64_t frames;               /* chunk length in frames */
} amx_chunk;

/* Loudness / finalize parameters (af_loudnorm linear mode + af_alimiter, :223). */
typedef struct amx_final_desc {
    double limit;                 /* 0.98 */
    double attack_ms;             /* 5 */
    double release_ms;            /* 50 */
    double level_in, level_out;   /* 1, 1 */
    int32_t auto_level;           /* 1 (alimiter default) */
    int32_t from_rest;            /* amx_finalize: != 0 -> every span starts from rest (its halo
                                   * ring, limiter idle) and d_lim_state is written, never read:
                                   * the speculative first run of a rank-to-rank hand-off (ABI 4) */
} amx_final_desc;

typedef struct amx_plan amx_plan;

typedef struct amx_plan_info {
    int64_t workspace_bytes;      /* caller-allocated device scratch for all calls */
    int64_t out_frames;           /* total output frames over all tracks of the plan */
    int32_t n_tracks;
    int32_t n_chunks;
    int64_t n_segments;           /* IIR segments over all chunks */
    int32_t seg_frames;           /* frames per IIR segment */
    int32_t scan_levels_eq;       /* scan window K (blocks of 16 segments) per filter */
    int32_t scan_levels_xover;
    int32_t scan_levels_kw;
    int32_t eq_dim;
    int32_t hop_frames;           /* libebur128 samples_in_100ms of the measurement stream */
    int32_t meas_rate;            /* the loudness measurement's rate: 192000 (see pass 1) */
    int32_t pad_;
    int64_t max_hops;             /* 100 ms hops of the longest track's measurement stream + 1:
                                     the d_hops row length amx_loudness_pass2 needs */
} amx_plan_info;

/* Per-track output span of this plan inside the full track timeline (for chunk
 * sharding over ranks: a rank holds a contiguous run of chunks of a track). */
typedef struct amx_track_span {
    int64_t out_offset;           /* first output frame of this plan's part, in the plan's d_out */
    int64_t out_frames;           /* frames this plan produces for the track */
    int64_t track_frame0;         /* index of that first frame in the WHOLE track timeline */
    int64_t track_frames_total;   /* output frames of the whole track (all ranks) */
} amx_track_span;

AMX_API int amx_abi_version(void);
AMX_API const char *amx_last_error(void);
/* Build provenance: the SHA-256 (hex) of the sources this library was compiled from
 * (csrc sources and headers, include/amx.h; amx/build.py source_hash), stamped at compile time.  The
 * Python binding refuses a library whose stamp differs from the tree it runs in. */
AMX_API const char *amx_build_id(void);

/* Build a plan (host only: designs nothing, derives scan matrices and segment
 * tables from the given coefficients, uploads small constant tables).
 * track_frame0/track_total may be NULL for a plan that holds whole tracks. */
AMX_API int amx_plan_create(const amx_chain_desc *desc, const amx_chunk *chunks, int32_t n_chunks,
                    const int64_t *track_frame0, const int64_t *track_total_frames,
                    int32_t seg_frames, amx_plan **out);
AMX_API void amx_plan_free(amx_plan *plan);
AMX_API int amx_plan_get_info(const amx_plan *plan, amx_plan_info *info);
AMX_API int amx_plan_track_span(const amx_plan *plan, int32_t track, amx_track_span *span);

/* Per-chunk chain: d_in float32 [frames, channels_in] -> d_out int16 [out_frames, 2]
 * (tracks back to back, chunks concatenated = the ffmpeg concat of :210-212). */
AMX_API int amx_run_chunks(amx_plan *plan, const float *d_in, int16_t *d_out, void *d_ws, void *stream);

/* The same chain one stage at a time (amx_run_chunks == stages 0..AMX_STAGE_COUNT-1 in
 * order), so a host can bracket individual kernels with events on its stream.
 * Stages that the settings make unnecessary are no-ops. */
#define AMX_STAGE_FRONT1 0   /* quantise + analog character + EQ zero-state GEMV */
#define AMX_STAGE_SCAN_EQ 1  /* affine scan -> exact EQ segment start states */
#define AMX_STAGE_FRONT2 2   /* EQ from true state + width -> int16 (+ crossover GEMV) */
#define AMX_STAGE_SCAN_XO 3  /* crossover scan */
#define AMX_STAGE_XOVER 4    /* crossover -> 3 int16 bands */
#define AMX_STAGE_RMS 5      /* exact audioop.rms detector per frame (block prefix sums) */
#define AMX_STAGE_ENV 6      /* envelope: speculation (every segment from a warmed-up guess) */
#define AMX_STAGE_FIX 7      /* envelope: parallel fix rounds + in-order exactness walk */
#define AMX_STAGE_APPLY 8    /* overlay of the gained bands -> chunk output */
#define AMX_STAGE_COUNT 9
AMX_API int amx_run_stage(amx_plan *plan, int32_t stage, const float *d_in, int16_t *d_out,
                          void *d_ws, void *stream);

/* Input decode (the s16 conversion of ffmpeg's segment split, :178, + pydub's
 * set_channels(2), :190): d_raw holds `frames` interleaved frames of `channels` (1 or
 * 2) samples in `format`; d_out [frames][2] int16 receives what the split's s16 WAV
 * chunks hold, mono duplicated to L = R.  (ABI 4) channels 3..8: d_out is int16
 * [frames][channels], no duplication (the input of amx_mc_run_chunks).  Asynchronous on
 * the stream.  A float32 file needs no call: amx_run_chunks quantises it (input_s16 = 0). */
#define AMX_PCM_U8 0      /* (v - 0x80) << 8 */
#define AMX_PCM_S16 1     /* v */
#define AMX_PCM_S24 2     /* 3-byte little-endian; v >> 8 */
#define AMX_PCM_S32 3     /* v >> 16 */
#define AMX_PCM_F32 4     /* clip(lrintf(v * 32768)) */
#define AMX_PCM_F64 5     /* clip(lrint(v * 32768)) */
/* big-endian PCM (AIFF / AIFF-C, the GUI's *.aiff, mastering_gui.py:170) and AIFF's
 * signed 8-bit: the same conversions after the byte swap; s8: v << 8 */
#define AMX_PCM_S8 6
#define AMX_PCM_S16BE 7
#define AMX_PCM_S24BE 8
#define AMX_PCM_S32BE 9
#define AMX_PCM_F32BE 10
#define AMX_PCM_F64BE 11
AMX_API int amx_pcm_to_s16(const void *d_raw, int64_t frames, int32_t channels, int32_t format,
                           int16_t *d_out, void *stream);

/* FLAC input (the GUI's *.flac, mastering_gui.py:170; ffmpeg decodes it at :178).  Host
 * decoder of the FLAC bitstream (RFC 9639), frames decoded on a thread pool (threads <= 0:
 * one per core).  amx_flac_decode writes out_frames x channels interleaved int32 samples,
 * left-justified to 32 bits (sample << (32 - bits_per_sample)) -- ffmpeg's decoded value,
 * which amx_pcm_to_s16 with AMX_PCM_S32 turns into the s16 chunk samples ffmpeg writes
 * (>> 16) -- and the frames decoded to *frames_out (out NULL: only *frames_out).  With
 * n_blocks, the FLAC frames' block sizes in stream order go to blocks[0 .. *n_blocks)
 * (blocks NULL: only the count): they are the packets whose start times the segment
 * split cuts at (:178).  Errors: AMX_EINVAL (not FLAC, a corrupt frame), AMX_ERANGE
 * (out_frames or max_blocks too small). */
typedef struct amx_flac_info_t {
    int32_t sample_rate, channels, bits_per_sample, max_block;
    int64_t total_frames;   /* STREAMINFO's total samples per channel (0: unknown) */
} amx_flac_info_t;
AMX_API int amx_flac_info(const uint8_t *data, int64_t size, amx_flac_info_t *info);
AMX_API int amx_flac_decode(const uint8_t *data, int64_t size, int32_t *out, int64_t out_frames,
                            int64_t *frames_out, int32_t threads, int32_t *blocks, int64_t max_blocks,
                            int64_t *n_blocks);

/* Diagnostics of the compressor envelope's fix-up (AMX_STAGE_FIX) of the last step run
 * on d_ws: out[0..3] = segments the chain walkers re-ran, the longest walk (segments one
 * wave re-ran in turn), chains, and segments of the optimistic parallel pass before them
 * (out[4..] are 0).  Synchronous (hipMemcpy): call it outside graph capture.  Replaces no
 * reference line. */
AMX_API int amx_env_counters(const amx_plan *plan, const void *d_ws, int32_t *out, int32_t n);

/* Gate a plan's per-sample kernels on a device word: with d_gate set, the K-weighting
 * passes (amx_loudness_pass1 / _pass2 at the plan's own rate) and amx_finalize's kernel
 * return at once unless (*d_gate >> 4) & 15 == 3 -- the chain track's k_decide mode
 * word says dynamic.  For the 192 kHz side plan of loudnorm's dynamic path held in a
 * captured step (MasteringJob.prepare_dynamic): a linear track's step then skips its
 * 192 kHz measurement passes and alimiter.  NULL removes the gate.  Replaces no
 * reference line (the reference only runs the 192 kHz pass 2 when it is needed, :240). */
AMX_API int amx_plan_set_gate(amx_plan *plan, const int32_t *d_gate);

/* Loudness pass 1 over d_out as ffmpeg's loudnorm pass 1 measures it (:229): with no
 * measured_* values af_loudnorm runs in dynamic mode, which takes 192 kHz input, so
 * the track is measured on libswresample's 192 kHz upsampling of it (recomputed on
 * the fly, never stored; libswresample's 1024-phase interpolating kernel where the
 * phase step is not an integer, 22.05 / 11.025 kHz) -- libebur128's
 * K filter, 400 ms / 3 s blocks and sample peak at 192 kHz.
 * K-filter zero-state GEMV per segment + exact scan + sample peaks.
 * d_edge [n_tracks][2][80][2] int16: the 80 output frames before and after a span
 * that does not start / end its track (the neighbour ranks' frames, which the
 * resampler's window reaches: 16 for the 32-tap upsampler, up to 67 for the longer
 * downsampling filters of inputs above 192 kHz); NULL when every span is a whole track.
 * d_kw_tail [n_tracks][2][4]: K-filter state at each span end assuming the span
 * started from rest (what the NEXT rank of a chunk-sharded track needs, see
 * amx_kw_propagate; NULL = not wanted, e.g. one GPU); d_peak [n_tracks][4]: per
 * channel the measured (192 kHz) stream's max |x| (loudnorm's input_tp), then
 * d_out's own max |x| (the limiter's input bound). */
AMX_API int amx_loudness_pass1(amx_plan *plan, const int16_t *d_out, const int16_t *d_edge,
                               double *d_kw_tail, double *d_peak, void *d_ws, void *stream);
/* amx_loudness_pass1 in its two launches (same arguments): part 0 = the one pass over
 * the samples (at 192 kHz: k_up, and k_up_edge beside it on the plan's second stream),
 * part 1 = peaks, scan, tails.  pass1 == part 0 then part 1; split so a caller can
 * time the sample pass alone. */
AMX_API int amx_loudness_pass1_part(amx_plan *plan, int32_t part, const int16_t *d_out,
                                    const int16_t *d_edge, double *d_kw_tail, double *d_peak,
                                    void *d_ws, void *stream);
/* af_loudnorm's 192 kHz modes (FFmpeg af_loudnorm.c; restated in oracle/amx_oracle.c
 * orc_loudnorm) on one whole track of the plan: the reference's pass 1 (:229) runs them
 * with the measured_* defaults (its JSON target_offset = target_i - the integrated
 * loudness of this output), and pass 2 (:240) runs them whenever the linear conditions
 * fail ("dynamic mode": 3 s look-ahead AGC smoothed over 100 ms frames, true-peak
 * limiter at target_tp, 192 kHz output).  A track shorter than 3 s takes af_loudnorm's
 * linear fallback (still at 192 kHz).  Options in dB as the reference passes them. */
typedef struct amx_loudnorm_desc {
    double target_i, target_lra, target_tp;                     /* I, LRA, TP */
    double measured_i, measured_lra, measured_tp, measured_thresh, offset;   /* pass 1: 0, 0, 99, -70, 0 */
    /* nonzero: d_ws2 still holds this track's 192 kHz stream and per-frame statistics from
     * the previous call on the same d_out, hop energies and scratch (pass 2 after pass 1:
     * the same input, resampled and measured the same way) -- neither is formed again;
     * 0: the call resamples d_out and forms them */
    int32_t reuse_stream;
} amx_loudnorm_desc;
/* output frames (ceil(frames * 192000 / fs)) and the d_ws2 bytes amx_loudnorm_192k needs */
AMX_API int amx_loudnorm_192k_size(const amx_plan *plan, int32_t track, int64_t *frames, int64_t *ws_bytes);
/* d_out: the plan's chain output (the track to normalise); d_hops / max_hops and d_peak:
 * amx_loudness_pass2's hop energies and amx_loudness_pass1's peaks of the same plan (the
 * 192 kHz stream's r128_in statistics); d_y192 [frames][2] s16: the output as the WAV
 * muxer writes it (av_clip_int16(llrint(x * 32768))); d_summary [16]: [0..1] = (1, offset)
 * when the < 3 s linear fallback ran, else (0, the final above_threshold).  Diagnostics:
 * on the frame-by-frame path (a quiet start) [2..9] = device cycles in the ring fills,
 * peak scans, envelopes, output, statistics and r128_out, then the peak-scan calls and
 * their serial chunks; on the parallel path [10..13] = segments re-run in order, FINAL
 * re-run (limiter active at its start), segments, hand-over to the frame-by-frame path. */
AMX_API int amx_loudnorm_192k(amx_plan *plan, int32_t track, const amx_loudnorm_desc *desc,
                              const int16_t *d_out, const double *d_hops, int64_t max_hops,
                              const double *d_peak, int16_t *d_y192, double *d_summary, void *d_ws2,
                              void *stream);
/* The same with the measured_* options and pass 1's target_offset read on the device,
 * so the whole dynamic path can be captured into one graph: d_measured (nullable) = a
 * k_decide statistics row of the track (amx_loudness_decide d_stats: [4] input_i, [7]
 * input_thresh, already the "%.2f" values pass 2 parses); d_offset_i (nullable) = the
 * statistics row of pass 1's output measurement ([0] its integrated loudness): offset =
 * "%.2f"(target_i - that) dB, as pass 1's JSON target_offset (:229-241).  A NULL
 * pointer takes desc's value.  d_gate (nullable) = the track's amx_loudness_decide
 * control word (d_ctl + track): unless it says dynamic mode, every kernel of the call
 * returns at once (a captured step then holds the dynamic path for the tracks that
 * need it). */
AMX_API int amx_loudnorm_192k_ex(amx_plan *plan, int32_t track, const amx_loudnorm_desc *desc,
                                 const double *d_measured, const double *d_offset_i,
                                 const int32_t *d_gate, const int16_t *d_out, const double *d_hops, int64_t max_hops,
                                 const double *d_peak, int16_t *d_y192, double *d_summary, void *d_ws2,
                                 void *stream);
/* A chunk-sharded track's share of one dynamic-mode filter run (:240 in dynamic mode on a
 * track split over ranks).  plan: a measure-only plan of the WHOLE track (d_out the whole
 * chain output, gathered from the ranks); every rank forms every frame's AGC gain from the
 * whole-track hop energies and runs the parallel form's segments [kb, ke) only; the
 * rank-to-rank hand-off is the limiter's true state at a segment boundary, one record of
 * rec_doubles doubles (amx_loudnorm_192k_segments).  part 0: the 192 kHz stream over
 * [u_lo, u_hi) (u_lo < 0: the range segments [kb, ke) read) and the frame statistics -- then read the int32 at ctl_offset of d_ws2: 0
 * means the parallel form runs, anything else (a quiet start, a track under 3 s) means the
 * whole track must run frame by frame (amx_loudnorm_192k_ex on one rank's whole data);
 * part 1: gains and the segments; part 2: the walk over [kb, ke) from d_rec_in (the true
 * state at kb, made by the previous rank's part 2; NULL on the rank holding segment 0),
 * which writes the true state at ke to d_rec_out (NULL on the last rank; a record whose
 * [7] is non-zero means the walk could not go on: the whole track must run frame by
 * frame).  Outputs: d_y192 frames [start(kb), start(ke)) (whole-track positions).
 * Replaces no single reference line: the reference runs the filter on one process. */
typedef struct amx_ln_shard {
    /* part 0: the 192 kHz stream over the window + every frame's statistics (control word 0:
     * the parallel form runs, 1: the track starts quietly or is under 3 s); 1: deltas,
     * gains, the fill pre-pass, segments [kb, ke) from guessed states; 2: the walk from the
     * true state at kb; (ABI 4) 3, on the rank with kb == 0 after part 0 said 1: a quiet
     * start's frames in order from the track start until the hand-over segment (control
     * words 4 / ho_k / ho_f, the deltas before ho_f written), or word 1 still when the track
     * stays quiet past segment ke - 1 -- the other ranks take the words and deltas from it.
     * windowed != 0: the rank holds only windows of the track (amx_loudnorm_192k_shard_window):
     * d_out = track frames [x_lo, x_hi), d_y192 = 192 kHz positions [y_lo, y_hi), d_ws2 of
     * the window's size with the stream u over [u_lo, u_hi) only (u_lo / u_hi ignored) */
    int32_t part, kb, ke, windowed;
    int64_t u_lo, u_hi;
    const double *d_rec_in;
    double *d_rec_out;
} amx_ln_shard;
AMX_API int amx_loudnorm_192k_shard(amx_plan *plan, int32_t track, const amx_loudnorm_desc *desc,
                                    const double *d_measured, const double *d_offset_i, const amx_ln_shard *sh,
                                    const int16_t *d_out, const double *d_hops, int64_t max_hops,
                                    const double *d_peak, int16_t *d_y192, double *d_summary, void *d_ws2,
                                    void *stream);
/* The windows a rank running segments [kb, ke) of the track's filter needs when it holds
 * no whole-track buffer (amx_ln_shard.windowed): win[0..1] = the chain-output frames
 * [x_lo, x_hi) its resampler reads (its own span plus halos of the neighbours' spans),
 * win[2..3] = the 192 kHz positions [u_lo, u_hi) its segments read, win[4..5] = the output
 * positions [y_lo, y_hi) they emit, win[6] = the byte offset in that d_ws2 of the int32
 * control words; (ABI 4: win holds 9) win[7] = the byte offset of the INNER frames' deltas
 * (win[8] = T doubles); *ws_bytes = the d_ws2 size of the window (the whole-track records stay;
 * the stream and the limiter waves are the window's).  Per-rank memory and traffic then
 * scale as 1 / ranks. */
AMX_API int amx_loudnorm_192k_shard_window(const amx_plan *plan, int32_t track, int32_t kb, int32_t ke,
                                           int64_t *win, int64_t *ws_bytes);
/* The parallel form's segments of the track's 192 kHz filter run: starts[k] (k < *K, cap
 * entries) = the output frame segment k starts at (starts[*K] = the frame count); *k_fin
 * = the first segment of the FINAL flush frame (one rank must hold [k_fin, K)); the
 * record size in doubles; the byte offset in d_ws2 of the int32 control words. */
AMX_API int amx_loudnorm_192k_segments(const amx_plan *plan, int32_t track, int64_t *starts, int32_t cap,
                                       int32_t *K, int32_t *k_fin, int32_t *rec_doubles, int64_t *ctl_offset);
/* Host helper for chunk-sharded tracks: out8 = A^frames * in8 (per channel 4x4 K-filter
 * transition at the measurement rate; frames of the measurement stream), so
 * carry(r+1) = A^{len_r} carry(r) + tail(r). */
AMX_API int amx_kw_propagate(const amx_plan *plan, int64_t frames, const double *in8, double *out8);
/* Loudness pass 2: K-filter from the exact state (d_kw_carry [n_tracks][2][4] = state
 * entering each span, NULL = rest: then the start states amx_loudness_pass1 left are
 * reused, so pass 1 must run first on the same d_ws), squared and summed per 100 ms hop on the
 * WHOLE-track hop grid: d_hops [n_tracks][max_hops][2] (zeroed here; hops a span only
 * partly covers hold partial sums -- sum them over ranks, e.g. RCCL all-reduce). */
AMX_API int amx_loudness_pass2(amx_plan *plan, const int16_t *d_out, const int16_t *d_edge,
                               const double *d_kw_carry, double *d_hops, int64_t max_hops,
                               void *d_ws, void *stream);
/* Gating-block (400 ms / 100 ms hop) and short-term (3 s / 1 s) histograms from
 * whole-track hop energies.  d_hist, d_st_hist [n_tracks][1000] uint64 (zeroed here). */
AMX_API int amx_loudness_histograms(amx_plan *plan, const double *d_hops, int64_t max_hops,
                            uint64_t *d_hist, uint64_t *d_st_hist, void *d_ws, void *stream);

/* alimiter geometry: ring size in samples (fs*attack*channels), the frame delay
 * (ring frames - 1 = halo frames a span needs from its predecessor) and the state
 * doubles per track for the general path. */
AMX_API int amx_limiter_geometry(const amx_plan *plan, const amx_final_desc *fd, int32_t *buffer_size,
                         int32_t *halo_frames, int64_t *state_doubles);
/* General-path alimiter scratch, plan-owned.  The span is cut into segments of
 * seg_frames frames (<= 0: 16384, or the last value set; >= 64 and >= the ring
 * frames); each segment warms up from the limiter's rest state over warm_frames
 * frames before it (< 0: 3 releases + the ring), runs in parallel, and an in-order
 * walk re-runs any segment whose guessed start state differs from the true one
 * (amx_final.hip).  Allocates device memory: call it before capturing
 * amx_finalize into a graph (amx_finalize calls it itself otherwise).  Replaces
 * no reference line: it sizes the parallel form of the alimiter at :223. */
AMX_API int amx_limiter_prepare(amx_plan *plan, const amx_final_desc *fd, int32_t seg_frames,
                                int32_t warm_frames);
/* Loudnorm decision on the device (af_loudnorm pass-1 statistics + pass-2 mode,
 * :229-242): per track, from the histograms and sample peak:
 *   d_stats [n_tracks][16] doubles: I, LRA, thresh, TP(dB), the same four after
 *     ffmpeg's "%.2f" print + parse, mode (0 off, 1 skip = silent, 2 linear,
 *     3 dynamic = unsupported), gain, limiter-idle flag, measured (192 kHz) sample
 *     peak, d_out's sample peak;
 *   d_peak [n_tracks][4] from amx_loudness_pass1;
 *   d_gains [n_tracks]: the linear gain, or -1 (no normalisation);
 *   d_ctl [n_tracks] int32: bit 0 = limiter provably idle (AMX_CTL_FAST), bits 4..7
 *     mode -- consumed by amx_finalize without a host round trip.
 * lufs_on = 0 (settings lufs None, :216) only computes the limiter flag. */
typedef struct amx_decide_desc {
    int32_t lufs_on, pad_;
    double target_i;              /* settings['lufs'] */
    double target_tp;             /* loudnorm TP=-1.5 (:229) */
    double target_lra;            /* loudnorm LRA=11 */
} amx_decide_desc;
#define AMX_CTL_FAST 1
AMX_API int amx_loudness_decide(amx_plan *plan, const amx_decide_desc *dd, const amx_final_desc *fd,
                                const uint64_t *d_hist, const uint64_t *d_st_hist, const double *d_peak,
                                double *d_stats, double *d_gains, int32_t *d_ctl, void *stream);
/* The n decision words d_ctl (amx_loudness_decide) stored into pinned host memory h_ctl
 * (hipHostMalloc'd, device-mapped) by a small kernel on the stream, with system-scope
 * stores: the host polls them while the step goes on (a captured step's host read,
 * without a copy node's completion stall).  Replaces no reference line: the reference
 * reads ffmpeg's printed statistics (:231-237). */
AMX_API int amx_publish_ctl(const int32_t *d_ctl, int32_t *h_ctl, int32_t n, void *stream);
/* The same words stored by amx_loudness_decide itself (its kernel's last stores; no node
 * of their own in a captured step): h_ctl = pinned host memory of n_tracks int32 words,
 * NULL to stop.  The plan keeps the pointer; the caller keeps the memory alive. */
AMX_API int amx_plan_set_publish(amx_plan *plan, int32_t *h_ctl);

/* Chunk-sharded tracks: K-filter state entering this plan's (single) span from the
 * zero-start tails of the n_prev spans before it.  Setup (host, once): frames_after[q]
 * = d_out frames between the end of span q and the start of this span (converted to
 * the measurement stream inside).  Then, on the
 * stream: d_carry [2][4] = sum_q A^{frames_after[q]} d_tails[q] (d_tails [n_prev][2][4]). */
AMX_API int amx_kw_carry_setup(amx_plan *plan, int32_t n_prev, const int64_t *frames_after);
AMX_API int amx_kw_carry(amx_plan *plan, const double *d_tails, double *d_carry, void *stream);
/* The same from the N > 1 step's gathered exchange rows in place (one kernel instead of
 * a copy, the carry and a max reduction): d_rows [world][ld] doubles, each rank's row =
 * its K-filter tail [2][4] at 0 and its sample peaks [4] at 8 (ld >= 12); d_carry as
 * above from the rows q < n_prev; d_peak [4] = the max over the world rows.  Replaces the
 * whole-file measurement's peaks of :229 (ebur128 over the concatenated track). */
AMX_API int amx_kw_carry_rows(amx_plan *plan, const double *d_rows, int32_t world, int32_t ld,
                              double *d_carry, double *d_peak, void *stream);

/* Finalize: loudnorm linear gain (d_gains[t] <= 0 -> no normalisation, :216) then
 * alimiter (:223) -> d_y int16 [out_frames, 2] (same frame indexing as d_x).
 * d_halo [n_tracks][halo_frames][2]: the input frames preceding each span (ignored
 * for spans that start their track).  Limiter path per track: with d_ctl (from
 * amx_loudness_decide) each track takes the path its AMX_CTL_FAST bit selects, on the
 * device; with d_ctl NULL, fast != 0 selects the idle path for every track.  The idle
 * path (max|gained sample| <= limit) is an exact delay + level; otherwise the
 * general limiter runs (parallel segments + in-order repair, bit-identical to the
 * sequential filter; scratch from amx_limiter_prepare), and d_lim_state
 * [n_tracks][state_doubles] carries its state in (span not starting the track) and out
 * (span end). */
AMX_API int amx_finalize(amx_plan *plan, const amx_final_desc *fd, const int16_t *d_x,
                 const double *d_gains, const int32_t *d_ctl, int32_t fast, const int16_t *d_halo,
                 int16_t *d_y, double *d_lim_state, void *d_ws, void *stream);

/* (ABI 4) The general limiter also writes every output frame's gain att (the value
 * its dst = delayed sample x att uses; 1 on idle stretches) to d_att [out_frames]
 * doubles, or stops (NULL).  The idle path (AMX_CTL_FAST) writes nothing: att = 1. */
AMX_API int amx_plan_set_limiter_trace(amx_plan *plan, double *d_att);

/* ---------------------------------------------------------------------------------
 * (ABI 4) Files with more than two channels (3..8).  The reference keeps such a chunk
 * as ONE interleaved 1-D stream (:252): analog character, EQ and crossover run along
 * it (:264-265, :274, :303), width leaves it alone (:268), pydub's compressor and
 * overlay work on frames of C samples (:306-309); ffmpeg's loudnorm measures the C
 * channels with libebur128's default channel map, and the alimiter's gain follows the
 * largest |sample| of each frame (:223).  The chain runs as pseudo-stereo sub-plans
 * (the stream in L) plus C-channel compressor kernels. */
typedef struct amx_mc_plan amx_mc_plan;
/* desc: the settings as for amx_plan_create, with channels_in = C (3..8) and
 * input_s16 saying what d_in holds (int16 or float32 [frames][C]); chunks in frames of
 * the C-channel input.  Replaces :185-214 for such a file. */
AMX_API int amx_mc_plan_create(const amx_chain_desc *desc, const amx_chunk *chunks, int32_t n_chunks,
                               int32_t seg_frames, amx_mc_plan **out);
AMX_API void amx_mc_plan_free(amx_mc_plan *plan);
/* workspace bytes for amx_mc_run_chunks, output frames (all chunks) */
AMX_API int amx_mc_plan_get_info(const amx_mc_plan *plan, int64_t *workspace_bytes, int64_t *out_frames);
/* the chunk chains of every chunk -> d_out int16 [out_frames][C] (the concat, :211) */
AMX_API int amx_mc_run_chunks(amx_mc_plan *plan, const void *d_in, int16_t *d_out, void *d_ws, void *stream);
/* loudnorm's measurement of a C-channel track, from a stereo measure plan run over the
 * channel pairs (0,1), (2,3), ... as tracks (the last pair of an odd C padded with a
 * silent channel): d_pairs int16 [ceil(C/2)][frames][2] from d_y int16 [frames][C] */
AMX_API int amx_mc_split_pairs(const int16_t *d_y, int64_t frames, int32_t channels, int16_t *d_pairs,
                               void *stream);
/* the pairs' hop energies [ceil(C/2)][max_hops][2] and peaks [ceil(C/2)][4] -> one
 * track's [max_hops][2] (sum over channels with libebur128's weights: 1 for L R C, 1.41
 * for the surrounds, 0 for unused channels; the second column 0) and peaks [4] (max) */
AMX_API int amx_mc_loudness_combine(const double *d_hops, int64_t max_hops, const double *d_peak,
                                    int32_t channels, double *d_hops1, double *d_peak1, void *stream);
/* the alimiter's peak signal: per frame the sample of the channel whose gained |value|
 * (d_gain[0]: loudnorm's linear gain, <= 0 none) is largest, in both channels of d_syn
 * int16 [frames][2] -- the limiter's state only ever sees per-frame peaks */
AMX_API int amx_mc_peak_pick(const int16_t *d_y, int64_t frames, int32_t channels, const double *d_gain,
                             int16_t *d_syn, void *stream);
/* the C-channel alimiter output from the peak signal's run (amx_finalize on a stereo
 * plan over d_syn with amx_plan_set_limiter_trace): out = limiter_out(gained sample
 * B - 1 frames earlier x att) per channel; d_ctl's AMX_CTL_FAST bit: att = 1 */
AMX_API int amx_mc_limiter_out(const amx_plan *plan, const amx_final_desc *fd, const int16_t *d_y,
                               int32_t channels, const double *d_gains, const int32_t *d_ctl,
                               const double *d_att, int16_t *d_out, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* AMX_H */
