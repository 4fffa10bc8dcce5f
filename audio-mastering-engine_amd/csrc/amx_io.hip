// amx_io.hip -- the input file's PCM -> the s16 stereo frames the chunk chain reads.
//
// The reference never sees the input's own sample format: ffmpeg's segment split
// (audio_mastering_engine.py:178) writes every chunk as a 16-bit PCM WAV (the wav
// muxer's default codec), converting with libswresample's audioconvert, and pydub
// then duplicates a mono chunk to stereo (set_channels(2), :190).  Restated per
// format (audioconvert.c CONV_FUNC, no dither -- swr's default):
//   u8  : (v - 0x80) << 8
//   s16 : v
//   s24 : decoded to s32 as v << 8, then >> 16          (= v >> 8, arithmetic)
//   s32 : v >> 16
//   f32 : av_clip_int16(lrintf(v * 32768))
//   f64 : av_clip_int16(lrint(v * 32768))
// AIFF / AIFF-C input (the GUI's *.aiff, mastering_gui.py:170): big-endian PCM and float
// take the same conversions after the byte swap (pcm_s16be ... pcm_f64be decode to the
// same sample formats); AIFF's 8-bit is signed (pcm_s8 decodes to u8 as v + 0x80, so
// the s16 value is v << 8).
// (float32 input normally skips this kernel: k_front1s quantises it in the chain's
// first pass.)  One thread per frame, grid-stride; a memory-bound pass.
#include "amx_dev.hpp"

namespace amx {

template <int FMT>
__device__ __forceinline__ int16_t pcm_sample(const uint8_t *__restrict__ raw, int64_t s) {
    if constexpr (FMT == AMX_PCM_U8) {
        return (int16_t)(((int)raw[s] - 0x80) * 256);
    } else if constexpr (FMT == AMX_PCM_S16) {
        return reinterpret_cast<const int16_t *>(raw)[s];
    } else if constexpr (FMT == AMX_PCM_S24) {
        const uint8_t *p = raw + 3 * s;
        const int v = (int)((uint32_t)p[0] << 8 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 24);
        return (int16_t)(v >> 16);
    } else if constexpr (FMT == AMX_PCM_S32) {
        return (int16_t)(reinterpret_cast<const int32_t *>(raw)[s] >> 16);
    } else if constexpr (FMT == AMX_PCM_F32) {
        return q_f32_to_s16_ffmpeg(reinterpret_cast<const float *>(raw)[s]);
    } else if constexpr (FMT == AMX_PCM_F64) {
        double v = rint(reinterpret_cast<const double *>(raw)[s] * 32768.0);
        v = fmin(fmax(v, -32768.0), 32767.0);
        return (int16_t)(int)v;
    } else if constexpr (FMT == AMX_PCM_S8) {
        return (int16_t)((int)(int8_t)raw[s] * 256);
    } else if constexpr (FMT == AMX_PCM_S16BE) {
        const uint8_t *p = raw + 2 * s;
        return (int16_t)(uint16_t)((uint32_t)p[0] << 8 | (uint32_t)p[1]);
    } else if constexpr (FMT == AMX_PCM_S24BE) {
        const uint8_t *p = raw + 3 * s;
        const int v = (int)((uint32_t)p[2] << 8 | (uint32_t)p[1] << 16 | (uint32_t)p[0] << 24);
        return (int16_t)(v >> 16);
    } else if constexpr (FMT == AMX_PCM_S32BE) {
        const uint8_t *p = raw + 4 * s;
        const int v = (int)((uint32_t)p[3] | (uint32_t)p[2] << 8 | (uint32_t)p[1] << 16 | (uint32_t)p[0] << 24);
        return (int16_t)(v >> 16);
    } else if constexpr (FMT == AMX_PCM_F32BE) {
        const uint8_t *p = raw + 4 * s;
        const uint32_t b = (uint32_t)p[3] | (uint32_t)p[2] << 8 | (uint32_t)p[1] << 16 | (uint32_t)p[0] << 24;
        return q_f32_to_s16_ffmpeg(__uint_as_float(b));
    } else {
        static_assert(FMT == AMX_PCM_F64BE, "PCM format");
        const uint8_t *p = raw + 8 * s;
        uint64_t b = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) b = b << 8 | (uint64_t)p[k];
        double v = rint(__longlong_as_double((long long)b) * 32768.0);
        v = fmin(fmax(v, -32768.0), 32767.0);
        return (int16_t)(int)v;
    }
}

template <int FMT, int CH>
__global__ void __launch_bounds__(AMX_BLOCK) k_pcm_to_s16(const uint8_t *__restrict__ raw,
                                                          int64_t frames,
                                                          uint32_t *__restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * AMX_BLOCK;
    for (int64_t i = (int64_t)blockIdx.x * AMX_BLOCK + threadIdx.x; i < frames; i += stride) {
        const int16_t l = pcm_sample<FMT>(raw, i * CH);
        const int16_t r = CH == 2 ? pcm_sample<FMT>(raw, i * CH + 1) : l;   // mono -> L = R (:190)
        out[i] = pack2(l, r);
    }
}

// a file with C > 2 channels: every sample to s16 in place of its layout ([frames][C],
// no duplication), what ffmpeg's split writes for it
template <int FMT>
__global__ void __launch_bounds__(AMX_BLOCK) k_pcm_to_s16_flat(const uint8_t *__restrict__ raw,
                                                               int64_t samples,
                                                               int16_t *__restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * AMX_BLOCK;
    for (int64_t i = (int64_t)blockIdx.x * AMX_BLOCK + threadIdx.x; i < samples; i += stride)
        out[i] = pcm_sample<FMT>(raw, i);
}

template <int FMT>
static hipError_t pcm_t(const uint8_t *raw, int64_t frames, int channels, uint32_t *out,
                        hipStream_t st) {
    const int64_t want = (frames + AMX_BLOCK - 1) / AMX_BLOCK;
    const unsigned g = (unsigned)(want < 8192 ? (want > 0 ? want : 1) : 8192);
    if (channels > 2) {
        const int64_t ns = frames * channels;
        const int64_t wf = (ns + AMX_BLOCK - 1) / AMX_BLOCK;
        const unsigned gf = (unsigned)(wf < 8192 ? (wf > 0 ? wf : 1) : 8192);
        hipLaunchKernelGGL(k_pcm_to_s16_flat<FMT>, dim3(gf), dim3(AMX_BLOCK), 0, st, raw, ns,
                           reinterpret_cast<int16_t *>(out));
    } else if (channels == 2)
        hipLaunchKernelGGL((k_pcm_to_s16<FMT, 2>), dim3(g), dim3(AMX_BLOCK), 0, st, raw, frames, out);
    else
        hipLaunchKernelGGL((k_pcm_to_s16<FMT, 1>), dim3(g), dim3(AMX_BLOCK), 0, st, raw, frames, out);
    return hipGetLastError();
}

hipError_t launch_pcm_to_s16(const void *raw, int64_t frames, int channels, int fmt, int16_t *out,
                             hipStream_t st) {
    if (frames <= 0) return hipSuccess;
    if (channels < 1 || channels > 8) return hipErrorInvalidValue;
    const uint8_t *r = reinterpret_cast<const uint8_t *>(raw);
    uint32_t *o = reinterpret_cast<uint32_t *>(out);
    switch (fmt) {
    case AMX_PCM_U8: return pcm_t<AMX_PCM_U8>(r, frames, channels, o, st);
    case AMX_PCM_S16: return pcm_t<AMX_PCM_S16>(r, frames, channels, o, st);
    case AMX_PCM_S24: return pcm_t<AMX_PCM_S24>(r, frames, channels, o, st);
    case AMX_PCM_S32: return pcm_t<AMX_PCM_S32>(r, frames, channels, o, st);
    case AMX_PCM_F32: return pcm_t<AMX_PCM_F32>(r, frames, channels, o, st);
    case AMX_PCM_F64: return pcm_t<AMX_PCM_F64>(r, frames, channels, o, st);
    case AMX_PCM_S8: return pcm_t<AMX_PCM_S8>(r, frames, channels, o, st);
    case AMX_PCM_S16BE: return pcm_t<AMX_PCM_S16BE>(r, frames, channels, o, st);
    case AMX_PCM_S24BE: return pcm_t<AMX_PCM_S24BE>(r, frames, channels, o, st);
    case AMX_PCM_S32BE: return pcm_t<AMX_PCM_S32BE>(r, frames, channels, o, st);
    case AMX_PCM_F32BE: return pcm_t<AMX_PCM_F32BE>(r, frames, channels, o, st);
    case AMX_PCM_F64BE: return pcm_t<AMX_PCM_F64BE>(r, frames, channels, o, st);
    default: return hipErrorInvalidValue;
    }
}

// Zero fill as a kernel node.  Every zeroing on a path that may be captured into a
// hipGraph goes through this instead of hipMemsetAsync: round 6 measured the runtime's
// fill node (a captured hipMemsetAsync) leaving a 1.2 KB counter array full of
// pointer-like words on the second replay of the dynamic path's graph (scripts/
// dyn_graph_probe.py, profiles/r06b_dyn_graph_probe.log), so the filter's boundary
// votes never matched and its walker re-ran 150 segments.
__global__ void __launch_bounds__(256) k_zero32(uint32_t *p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = 0u;
}

// ----------------------------------------- more than two channels (round 6)
// The C-channel file as ONE interleaved stream (:252) in the L channel of pseudo-stereo
// int16 pairs (R = 0): stream sample q = input sample q.  float32 input takes ffmpeg's
// s16 conversion (A.1) per sample.
__global__ void __launch_bounds__(256) k_mc_pack(const void *__restrict__ in, int64_t samples, int in_s16,
                                                 uint32_t *__restrict__ pairs) {
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < samples; q += (int64_t)gridDim.x * 256) {
        const int16_t v = in_s16 ? reinterpret_cast<const int16_t *>(in)[q]
                                 : q_f32_to_s16_ffmpeg(reinterpret_cast<const float *>(in)[q]);
        pairs[q] = (uint32_t)(uint16_t)v;
    }
}
__global__ void __launch_bounds__(256) k_mc_unpack(const uint32_t *__restrict__ pairs, int64_t samples,
                                                   int16_t *__restrict__ out) {
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < samples; q += (int64_t)gridDim.x * 256)
        out[q] = (int16_t)(uint16_t)(pairs[q] & 0xffffu);
}
// channel pairs (0,1), (2,3), ... of y [frames][C] as stereo tracks [P][frames][2]
__global__ void __launch_bounds__(256) k_mc_split_pairs(const int16_t *__restrict__ y, int64_t frames, int C,
                                                        int16_t *__restrict__ pairs) {
    const int P = (C + 1) / 2;
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < frames * P; q += (int64_t)gridDim.x * 256) {
        const int p = (int)(q / frames);
        const int64_t f = q - (int64_t)p * frames;
        const int16_t l = y[f * C + 2 * p];
        const int16_t r = 2 * p + 1 < C ? y[f * C + 2 * p + 1] : (int16_t)0;
        reinterpret_cast<uint32_t *>(pairs)[q] = pack2(l, r);
    }
}
// libebur128's default channel map (ebur128_init_channel_map): 4 channels L R Ls Rs, 5
// L R C Ls Rs, otherwise L R C unused Ls Rs, later channels unused; the surrounds
// (Mp110 / Mm110) weigh 1.41 (ebur128_calc_gating_block)
__device__ __forceinline__ double ebur_weight(int C, int c) {
    if (C == 4) return c < 2 ? 1.0 : 1.41;
    if (C == 5) return c < 3 ? 1.0 : 1.41;
    return c < 3 ? 1.0 : (c == 3 ? 0.0 : (c < 6 ? 1.41 : 0.0));
}
__global__ void __launch_bounds__(256) k_mc_loudness_combine(const double *__restrict__ hops, int64_t max_hops,
                                                             const double *__restrict__ peak, int C,
                                                             double *__restrict__ hops1, double *__restrict__ peak1) {
    const int P = (C + 1) / 2;
    for (int64_t h = (int64_t)blockIdx.x * 256 + threadIdx.x; h < max_hops; h += (int64_t)gridDim.x * 256) {
        double sum = 0.0;
        for (int c = 0; c < C; c++) {
            const double w = ebur_weight(C, c);
            if (w == 0.0) continue;                           // FF_EBUR128_UNUSED
            double e = hops[((int64_t)(c >> 1) * max_hops + h) * 2 + (c & 1)];
            if (w != 1.0) e *= w;
            sum += e;
        }
        hops1[2 * h] = sum;
        hops1[2 * h + 1] = 0.0;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        double m192 = 0.0, mout = 0.0;
        for (int p = 0; p < P; p++) {
            m192 = fmax(m192, fmax(peak[4 * p], peak[4 * p + 1]));
            mout = fmax(mout, fmax(peak[4 * p + 2], peak[4 * p + 3]));
        }
        peak1[0] = peak1[1] = m192;
        peak1[2] = peak1[3] = mout;
    }
}

static dim3 grid_stride(int64_t n) {
    const int64_t g = (n + 255) / 256;
    return dim3((unsigned)(g < 4096 ? (g > 0 ? g : 1) : 4096));
}
hipError_t launch_mc_pack(const void *in, int64_t samples, int in_s16, uint32_t *pairs, hipStream_t st) {
    if (samples <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_mc_pack, grid_stride(samples), dim3(256), 0, st, in, samples, in_s16, pairs);
    return hipGetLastError();
}
hipError_t launch_mc_unpack(const uint32_t *pairs, int64_t samples, int16_t *out, hipStream_t st) {
    if (samples <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_mc_unpack, grid_stride(samples), dim3(256), 0, st, pairs, samples, out);
    return hipGetLastError();
}
hipError_t launch_mc_split_pairs(const int16_t *y, int64_t frames, int C, int16_t *pairs, hipStream_t st) {
    if (frames <= 0) return hipSuccess;
    if (C < 1 || C > 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_mc_split_pairs, grid_stride(frames * ((C + 1) / 2)), dim3(256), 0, st, y, frames, C, pairs);
    return hipGetLastError();
}
hipError_t launch_mc_loudness_combine(const double *hops, int64_t max_hops, const double *peak, int C,
                                      double *hops1, double *peak1, hipStream_t st) {
    if (C < 1 || C > 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_mc_loudness_combine, grid_stride(max_hops), dim3(256), 0, st, hops, max_hops, peak, C,
                       hops1, peak1);
    return hipGetLastError();
}

hipError_t launch_zero(void *p, size_t bytes, hipStream_t st) {
    if (bytes == 0) return hipSuccess;
    if (!p || (bytes & 3) || (reinterpret_cast<uintptr_t>(p) & 3)) return hipErrorInvalidValue;
    const int64_t n = (int64_t)(bytes / 4);
    const int64_t g = (n + 255) / 256;
    hipLaunchKernelGGL(k_zero32, dim3((unsigned)(g < 1024 ? g : 1024)), dim3(256), 0, st,
                       reinterpret_cast<uint32_t *>(p), n);
    return hipGetLastError();
}

}  // namespace amx
