// amx_flac.cpp -- FLAC input (the GUI's *.flac, mastering_gui.py:170; ffmpeg decodes it at
// audio_mastering_engine.py:178 before the segment muxer writes s16 WAV chunks).
//
// A host decoder of the FLAC bitstream (RFC 9639): STREAMINFO, frame headers (CRC-8),
// CONSTANT / VERBATIM / FIXED / LPC subframes with wasted bits, partitioned Rice residuals
// (4- and 5-bit parameters, escapes), the three stereo decorrelations, frame CRC-16.
// Frames are independent: the decoder finds every frame start (sync code + a header whose
// CRC-8 matches), decodes candidate frames on a thread pool, and keeps the chain that
// tiles the stream from the first frame (a false sync inside frame data fails its CRC-16
// or is not reached by the chain).  Output: interleaved int32 samples left-justified to
// 32 bits -- what ffmpeg's decoder hands on for depths above 16 (AV_SAMPLE_FMT_S32,
// sample << (32 - bps)); for depths up to 16 it hands on s16 (sample << (16 - bps)), the
// same value after the s32 -> s16 conversion (>> 16) the device decode applies
// (amx_pcm_to_s16, AMX_PCM_S32).  So a FLAC file reaches the chain as the s16 chunks
// ffmpeg would write.
#include "../../include/amx.h"

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

// MSB-first bit reader over a 64-bit cache refilled a byte at a time; reads past the
// end set `bad` and return zeros
struct BitReader {
    const uint8_t *p;
    int64_t n;          // bytes
    int64_t byte;       // next byte to load into the cache
    uint64_t cache = 0; // valid bits left-aligned
    int nb = 0;         // valid bits in the cache
    bool bad = false;
    BitReader(const uint8_t *d, int64_t size, int64_t byte0) : p(d), n(size), byte(byte0) {}
    int64_t pos() const { return byte * 8 - nb; }                 // bit position
    void seek(int64_t bitpos) {
        byte = bitpos >> 3;
        cache = 0;
        nb = 0;
        const int skip = (int)(bitpos & 7);
        if (skip) bits(skip);
    }
    void refill() {
        while (nb <= 56) {
            if (byte >= n) {
                if (nb == 0) bad = true;
                return;
            }
            cache |= (uint64_t)p[byte++] << (56 - nb);
            nb += 8;
        }
    }
    uint64_t bits(int k) {   // k <= 56 per call; larger requests are split
        if (k == 0) return 0;
        if (k > 32) {
            const uint64_t hi = bits(k - 32);
            return (hi << 32) | bits(32);
        }
        if (nb < k) {
            refill();
            if (nb < k) { bad = true; nb = 0; cache = 0; return 0; }
        }
        const uint64_t v = cache >> (64 - k);
        cache <<= k;
        nb -= k;
        return v;
    }
    uint32_t bit() { return (uint32_t)bits(1); }
    int64_t sbits(int k) {   // two's complement, k in 0..64
        if (k == 0) return 0;
        const uint64_t v = bits(k);
        if (k == 64) return (int64_t)v;
        const uint64_t sign = 1ull << (k - 1);
        return (int64_t)((v ^ sign) - sign);
    }
    uint32_t unary() {       // zeros before the next 1 (which is consumed)
        uint32_t q = 0;
        for (;;) {
            if (nb == 0) {
                refill();
                if (nb == 0) { bad = true; return q; }
            }
            if (cache == 0) {   // all valid bits zero
                q += (uint32_t)nb;
                nb = 0;
                continue;
            }
            const int z = __builtin_clzll(cache);
            if (z >= nb) {
                q += (uint32_t)nb;
                nb = 0;
                cache = 0;
                continue;
            }
            q += (uint32_t)z;
            cache = z + 1 < 64 ? cache << (z + 1) : 0;
            nb -= z + 1;
            return q;
        }
    }
    void align() { seek((pos() + 7) & ~int64_t(7)); }
};

// table-driven CRC-8 (poly 0x07) and CRC-16 (poly 0x8005), MSB first, initial 0
struct CrcTables {
    uint8_t t8[256];
    uint16_t t16[256];
    CrcTables() {
        for (int i = 0; i < 256; i++) {
            uint8_t c = (uint8_t)i;
            for (int k = 0; k < 8; k++) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : (c << 1));
            t8[i] = c;
            uint16_t w = (uint16_t)(i << 8);
            for (int k = 0; k < 8; k++) w = (uint16_t)((w & 0x8000) ? (w << 1) ^ 0x8005 : (w << 1));
            t16[i] = w;
        }
    }
};
const CrcTables &crc_tables() {
    static const CrcTables t;
    return t;
}

uint8_t crc8(const uint8_t *d, int64_t n) {
    const CrcTables &T = crc_tables();
    uint8_t c = 0;
    for (int64_t i = 0; i < n; i++) c = T.t8[c ^ d[i]];
    return c;
}

uint16_t crc16(const uint8_t *d, int64_t n) {
    const CrcTables &T = crc_tables();
    uint16_t c = 0;
    for (int64_t i = 0; i < n; i++) c = (uint16_t)((c << 8) ^ T.t16[(c >> 8) ^ d[i]]);
    return c;
}

struct StreamInfo {
    int rate = 0, channels = 0, bps = 0, max_block = 0;
    int64_t max_frame = 0;     // STREAMINFO's largest frame in bytes (0: unknown)
    int64_t total = 0;
    int64_t first_frame = 0;   // byte offset of the first frame
};

int parse_streaminfo(const uint8_t *d, int64_t n, StreamInfo &si) {
    if (n < 42 || std::memcmp(d, "fLaC", 4) != 0) return AMX_EINVAL;
    int64_t pos = 4;
    bool have = false;
    for (;;) {
        if (pos + 4 > n) return AMX_EINVAL;
        const int last = d[pos] >> 7, type = d[pos] & 0x7f;
        const int64_t len = ((int64_t)d[pos + 1] << 16) | (d[pos + 2] << 8) | d[pos + 3];
        if (pos + 4 + len > n) return AMX_EINVAL;
        if (type == 0) {
            if (len < 34) return AMX_EINVAL;
            BitReader br(d, n, pos + 4);
            br.bits(16);                                   // min block size
            si.max_block = (int)br.bits(16);
            br.bits(24);                                   // min frame size
            si.max_frame = (int64_t)br.bits(24);
            si.rate = (int)br.bits(20);
            si.channels = (int)br.bits(3) + 1;
            si.bps = (int)br.bits(5) + 1;
            si.total = (int64_t)br.bits(36);
            have = true;
        }
        pos += 4 + len;
        if (last) break;
    }
    if (!have || si.rate <= 0 || si.bps < 4 || si.bps > 32) return AMX_EINVAL;
    si.first_frame = pos;
    return AMX_OK;
}

struct FrameHdr {
    int block = 0, channels = 0, assign = 0, bps = 0;
    int64_t data_bit = 0;   // bit position of the first subframe
};

// the frame header at byte b (sync, fields, CRC-8); false: not a frame start
bool parse_header(const uint8_t *d, int64_t n, int64_t b, const StreamInfo &si, FrameHdr &h) {
    if (b + 6 > n || d[b] != 0xFF || (d[b + 1] & 0xFE) != 0xF8) return false;
    BitReader br(d, n, b);
    br.bits(15);
    br.bits(1);                                            // blocking strategy
    const int bs = (int)br.bits(4), sr = (int)br.bits(4);
    const int ca = (int)br.bits(4), ss = (int)br.bits(3);
    if (br.bits(1) != 0 || bs == 0 || sr == 15 || ca > 10 || ss == 3) return false;
    // coded frame / sample number (UTF-8-like, up to 7 bytes)
    const uint32_t b0 = (uint32_t)br.bits(8);
    int extra = 0;
    if (b0 < 0x80) extra = 0;
    else if ((b0 & 0xE0) == 0xC0) extra = 1;
    else if ((b0 & 0xF0) == 0xE0) extra = 2;
    else if ((b0 & 0xF8) == 0xF0) extra = 3;
    else if ((b0 & 0xFC) == 0xF8) extra = 4;
    else if ((b0 & 0xFE) == 0xFC) extra = 5;
    else if (b0 == 0xFE) extra = 6;
    else return false;
    for (int i = 0; i < extra; i++)
        if ((br.bits(8) & 0xC0) != 0x80) return false;
    int block;
    if (bs == 1) block = 192;
    else if (bs <= 5) block = 576 << (bs - 2);
    else if (bs == 6) block = (int)br.bits(8) + 1;
    else if (bs == 7) block = (int)br.bits(16) + 1;
    else block = 256 << (bs - 8);
    if (sr == 12) br.bits(8);
    else if (sr == 13 || sr == 14) br.bits(16);
    if (br.bad) return false;
    const int64_t hb = br.pos() >> 3;                      // header bytes before the CRC
    if (hb >= n || crc8(d + b, hb - b) != d[hb]) return false;
    static const int ss_bits[8] = {0, 8, 12, 0, 16, 20, 24, 32};
    h.block = block;
    h.assign = ca;
    h.channels = ca < 8 ? ca + 1 : 2;
    h.bps = ss == 0 ? si.bps : ss_bits[ss];
    h.data_bit = (hb + 1) * 8;
    return h.channels == si.channels;
}

// Rice-coded residual of a subframe into res[order .. block)
bool residual(BitReader &br, int block, int order, int64_t *res) {
    const int method = (int)br.bits(2);
    if (method > 1) return false;
    const int pbits = method == 0 ? 4 : 5, esc = (1 << pbits) - 1;
    const int porder = (int)br.bits(4);
    const int parts = 1 << porder;
    if ((block >> porder) < order || (block & (parts - 1)) != 0) return false;
    int64_t i = order;
    for (int p = 0; p < parts; p++) {
        const int64_t cnt = (block >> porder) - (p == 0 ? order : 0);
        const int k = (int)br.bits(pbits);
        if (k == esc) {
            const int nb = (int)br.bits(5);
            for (int64_t j = 0; j < cnt; j++) res[i++] = br.sbits(nb);
        } else {
            for (int64_t j = 0; j < cnt; j++) {
                const uint64_t q = br.unary();
                const uint64_t u = (q << k) | br.bits(k);
                res[i++] = (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
            }
        }
        if (br.bad) return false;
    }
    return true;
}

// one subframe of `block` samples at sample depth bps into s
bool subframe(BitReader &br, int block, int bps, int64_t *s) {
    if (br.bit() != 0) return false;
    const int type = (int)br.bits(6);
    int wasted = 0;
    if (br.bit()) wasted = (int)br.unary() + 1;
    if (wasted >= bps) return false;
    const int eb = bps - wasted;
    if (type == 0) {
        const int64_t v = br.sbits(eb);
        for (int i = 0; i < block; i++) s[i] = v;
    } else if (type == 1) {
        for (int i = 0; i < block; i++) s[i] = br.sbits(eb);
    } else if (type >= 8 && type <= 12) {
        const int order = type - 8;
        if (order > block) return false;
        for (int i = 0; i < order; i++) s[i] = br.sbits(eb);
        if (!residual(br, block, order, s)) return false;
        // the predictors in wrapping uint64 arithmetic: a hostile stream's residuals can
        // push them past int64 (undefined for signed); a valid stream never wraps.
        // Order 0 predicts 0: the samples are the residuals (and s[i - 1] would read
        // before the subframe at i = 0 -- found by the host ASan build, test_sanitize.py)
        if (order > 0)
            for (int i = order; i < block; i++) {
                uint64_t pred = 0;
                const uint64_t a = (uint64_t)s[i - 1];
                switch (order) {
                case 1: pred = a; break;
                case 2: pred = 2 * a - (uint64_t)s[i - 2]; break;
                case 3: pred = 3 * a - 3 * (uint64_t)s[i - 2] + (uint64_t)s[i - 3]; break;
                case 4: pred = 4 * a - 6 * (uint64_t)s[i - 2] + 4 * (uint64_t)s[i - 3] - (uint64_t)s[i - 4]; break;
                default: break;
                }
                s[i] = (int64_t)((uint64_t)s[i] + pred);
            }
    } else if (type >= 32) {
        const int order = type - 31;
        if (order > block) return false;
        for (int i = 0; i < order; i++) s[i] = br.sbits(eb);
        const int prec = (int)br.bits(4) + 1;
        if (prec == 16) return false;
        const int shift = (int)br.sbits(5);
        if (shift < 0) return false;
        int64_t c[32];
        for (int i = 0; i < order; i++) c[i] = br.sbits(prec);
        if (!residual(br, block, order, s)) return false;
        for (int i = order; i < block; i++) {
            uint64_t acc = 0;                           // wrapping, as above
            for (int k = 0; k < order; k++) acc += (uint64_t)c[k] * (uint64_t)s[i - 1 - k];
            s[i] = (int64_t)((uint64_t)s[i] + (uint64_t)((int64_t)acc >> shift));
        }
    } else {
        return false;
    }
    if (wasted)
        for (int i = 0; i < block; i++) s[i] = (int64_t)((uint64_t)s[i] << wasted);
    return !br.bad;
}

struct Decoded {
    bool ok = false;
    int block = 0;
    int64_t end = 0;   // byte after the frame (CRC-16 included)
    std::vector<int32_t> pcm;   // block x channels, when kept
};

// decode the frame at byte b into out (block x channels interleaved, left-justified int32)
Decoded decode_frame(const uint8_t *d, int64_t n, int64_t b, const StreamInfo &si, std::vector<int64_t> &tmp,
                     int32_t *out, int64_t out_cap) {
    Decoded r;
    FrameHdr h;
    if (!parse_header(d, n, b, si, h)) return r;
    const int B = h.block, C = h.channels;
    tmp.resize((size_t)B * C);
    // a frame is never longer than STREAMINFO's largest frame, or (unknown) than twice its
    // verbatim size: the bound stops a false sync's "frame" from decoding the rest of the
    // file as residuals
    const int64_t lim = si.max_frame > 0 ? si.max_frame
                                         : 2 * ((int64_t)B * C * (h.bps + 1) / 8) + 1024;
    n = std::min<int64_t>(n, b + lim);
    BitReader br(d, n, 0);
    br.seek(h.data_bit);
    for (int c = 0; c < C; c++) {
        // the side channel carries one more bit (left/side: 1, side/right: 0, mid/side: 1)
        const bool side = (h.assign == 8 && c == 1) || (h.assign == 9 && c == 0) || (h.assign == 10 && c == 1);
        if (!subframe(br, B, h.bps + (side ? 1 : 0), tmp.data() + (size_t)c * B)) return r;
    }
    br.align();
    const int64_t cb = br.pos() >> 3;
    if (cb + 2 > n) return r;
    if (crc16(d + b, cb - b) != (uint16_t)((d[cb] << 8) | d[cb + 1])) return r;
    r.end = cb + 2;
    r.block = B;
    r.ok = true;
    if (!out) return r;
    if ((int64_t)B * C > out_cap) { r.ok = false; return r; }
    const int sh = 32 - h.bps;
    int64_t *s0 = tmp.data(), *s1 = tmp.data() + B;
    for (int i = 0; i < B; i++) {
        int64_t v[8];
        for (int c = 0; c < C; c++) v[c] = tmp[(size_t)c * B + i];
        if (h.assign == 8) { v[1] = s0[i] - s1[i]; }                 // left, side -> right
        else if (h.assign == 9) { v[0] = s0[i] + s1[i]; }            // side, right -> left
        else if (h.assign == 10) {                                   // mid, side
            const int64_t m = (int64_t)((uint64_t)s0[i] << 1) | (s1[i] & 1);
            v[0] = (m + s1[i]) >> 1;
            v[1] = (m - s1[i]) >> 1;
        }
        for (int c = 0; c < C; c++) out[(int64_t)i * C + c] = (int32_t)(uint32_t)((uint64_t)v[c] << sh);
    }
    return r;
}

}  // namespace

extern "C" {

AMX_API int amx_flac_info(const uint8_t *data, int64_t size, amx_flac_info_t *info) {
    if (!data || !info) return AMX_EINVAL;
    StreamInfo si;
    const int rc = parse_streaminfo(data, size, si);
    if (rc != AMX_OK) return rc;
    info->sample_rate = si.rate;
    info->channels = si.channels;
    info->bits_per_sample = si.bps;
    info->total_frames = si.total;
    info->max_block = si.max_block;
    return AMX_OK;
}

AMX_API int amx_flac_decode(const uint8_t *data, int64_t size, int32_t *out, int64_t out_frames,
                            int64_t *frames_out, int32_t threads, int32_t *blocks, int64_t max_blocks,
                            int64_t *n_blocks) {
    if (!data || !frames_out) return AMX_EINVAL;
    StreamInfo si;
    int rc = parse_streaminfo(data, size, si);
    if (rc != AMX_OK) return rc;
    const int C = si.channels;
    // frame starts: every sync whose header parses with a matching CRC-8
    std::vector<int64_t> cand;
    for (int64_t b = si.first_frame; b + 1 < size; b++) {
        if (data[b] != 0xFF || (data[b + 1] & 0xFE) != 0xF8) continue;
        FrameHdr h;
        if (parse_header(data, size, b, si, h)) cand.push_back(b);
    }
    if (cand.empty() || cand[0] != si.first_frame) {
        *frames_out = 0;
        return si.total == 0 && cand.empty() ? AMX_OK : AMX_EINVAL;
    }
    // decode every candidate in parallel (keeping the samples unless this is a size query)
    const int64_t nc = (int64_t)cand.size();
    std::vector<Decoded> dec((size_t)nc);
    int nt = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
    nt = (int)std::min<int64_t>(nt, std::max<int64_t>(1, nc / 4));
    std::atomic<int64_t> next{0};
    const bool keep = out != nullptr;
    auto pass = [&]() {
        std::vector<int64_t> tmp;
        for (;;) {
            const int64_t i = next.fetch_add(4);
            if (i >= nc) break;
            for (int64_t k = i; k < std::min(nc, i + 4); k++) {
                Decoded &r = dec[(size_t)k];
                FrameHdr h;
                if (keep && parse_header(data, size, cand[(size_t)k], si, h)) {
                    r.pcm.resize((size_t)h.block * C);
                    const Decoded q = decode_frame(data, size, cand[(size_t)k], si, tmp, r.pcm.data(),
                                                   (int64_t)h.block * C);
                    r.ok = q.ok;
                    r.block = q.block;
                    r.end = q.end;
                    if (!r.ok) std::vector<int32_t>().swap(r.pcm);
                } else {
                    r = decode_frame(data, size, cand[(size_t)k], si, tmp, nullptr, 0);
                }
            }
        }
    };
    {
        std::vector<std::thread> pool;
        for (int t = 1; t < nt; t++) pool.emplace_back(pass);
        pass();
        for (auto &th : pool) th.join();
    }
    // the chain of frames that tiles the stream from the first frame
    std::vector<int64_t> chain, first_sample;
    int64_t k = 0, samples = 0;
    while (k < nc && dec[(size_t)k].ok) {
        chain.push_back(k);
        first_sample.push_back(samples);
        samples += dec[(size_t)k].block;
        const int64_t e = dec[(size_t)k].end;
        if (e >= size) break;
        const auto it = std::lower_bound(cand.begin(), cand.end(), e);
        if (it == cand.end() || *it != e) break;
        k = it - cand.begin();
    }
    if (si.total > 0 && samples > si.total) samples = si.total;   // (a padded last frame)
    // a frame that fails its CRC-16 (or a truncated file) ends the chain early: refused,
    // rather than handing on a shortened track
    if (si.total > 0 && samples < si.total) return AMX_EINVAL;
    if (n_blocks) {                                              // the packets (frames) in order
        *n_blocks = (int64_t)chain.size();
        if (blocks) {
            if ((int64_t)chain.size() > max_blocks) return AMX_ERANGE;
            for (size_t q = 0; q < chain.size(); q++) blocks[q] = dec[(size_t)chain[q]].block;
        }
    }
    if (!out) {                                                  // size query
        *frames_out = samples;
        return AMX_OK;
    }
    if (samples > out_frames) return AMX_ERANGE;
    // the chain's samples into the caller's buffer
    std::atomic<int64_t> nx{0};
    auto copy = [&]() {
        for (;;) {
            const int64_t q = nx.fetch_add(1);
            if (q >= (int64_t)chain.size()) break;
            const int64_t f0 = first_sample[(size_t)q];
            const Decoded &r = dec[(size_t)chain[(size_t)q]];
            const int64_t take = std::min<int64_t>(r.block, samples - f0);
            if (take > 0) std::memcpy(out + f0 * C, r.pcm.data(), (size_t)take * C * sizeof(int32_t));
        }
    };
    {
        std::vector<std::thread> pool;
        for (int t = 1; t < nt; t++) pool.emplace_back(copy);
        copy();
        for (auto &th : pool) th.join();
    }
    *frames_out = samples;
    return AMX_OK;
}

}  // extern "C"
