// FLAC decode on the host (C ABI aa_flac_*), for load_recording
// (src/identify_tracks.py:49-62), which hands every file to ffmpeg through
// audioread.  The bitstream is the one RFC 9639 specifies: metadata blocks
// after "fLaC" (an ID3v2 tag in front is skipped), then frames of up to 8
// channels, each channel a CONSTANT / VERBATIM / FIXED (order 0-4) / LPC
// (order 1-32) subframe with optional wasted bits and a partitioned Rice
// residual (4- or 5-bit parameters, escape partitions), stereo decorrelated
// as left/side, side/right or mid/side.  Frame headers are checked against
// their CRC-8 and whole frames against their CRC-16; a damaged frame is an
// error (the reference turns any decode failure into "Could not load").
//
// Output is the decoded integer samples, interleaved, at the stream's own bit
// depth; the s16 conversion ffmpeg applies before librosa sees the samples
// (left-justify into s16 / s32, then s32 -> s16 by >> 16) is done by the
// caller (aa_amd/audio.py) exactly as for WAV.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "aa_common.h"

namespace {

using aa::set_error;

struct BitReader {
    const uint8_t* p;
    size_t n;       // bytes
    uint64_t pos;   // bit position

    uint64_t be64(size_t byte) const {
        if (byte + 8 <= n) {
            uint64_t v;
            memcpy(&v, p + byte, 8);
            return __builtin_bswap64(v);
        }
        uint64_t v = 0;
        for (size_t i = 0; i < 8; ++i) v = (v << 8) | (byte + i < n ? p[byte + i] : 0);
        return v;
    }
    // k in [0, 32]
    uint32_t get(int k) {
        if (k == 0) return 0;
        const uint64_t v = be64(pos >> 3) << (pos & 7);  // >= 57 valid bits
        pos += k;
        return (uint32_t)(v >> (64 - k));
    }
    int64_t get_signed(int k) {  // k in [0, 33]
        if (k == 0) return 0;
        uint64_t u;
        if (k > 32) {
            u = (uint64_t)get(k - 32) << 32;
            u |= get(32);
        } else {
            u = get(k);
        }
        return (int64_t)(u << (64 - k)) >> (64 - k);
    }
    // zeros before the next 1 bit (the 1 is consumed); false past the end
    bool unary(uint32_t& q) {
        uint32_t z = 0;
        for (;;) {
            if (pos >= (uint64_t)n * 8) return false;
            const uint64_t v = be64(pos >> 3) << (pos & 7);
            const int valid = 64 - (int)(pos & 7);
            if (v == 0) {
                z += valid;
                pos += valid;
                continue;
            }
            const int c = __builtin_clzll(v);
            z += c;
            pos += c + 1;
            q = z;
            return true;
        }
    }
    bool overrun() const { return pos > (uint64_t)n * 8; }
    void align() { pos = (pos + 7) & ~(uint64_t)7; }
};

uint8_t crc8(const uint8_t* d, size_t len) {  // x^8 + x^2 + x + 1
    uint8_t c = 0;
    for (size_t i = 0; i < len; ++i) {
        c ^= d[i];
        for (int b = 0; b < 8; ++b) c = (c & 0x80) ? (uint8_t)((c << 1) ^ 0x07) : (uint8_t)(c << 1);
    }
    return c;
}

struct Crc16Table {
    uint16_t t[256];
    Crc16Table() {
        for (int i = 0; i < 256; ++i) {
            uint16_t c = (uint16_t)(i << 8);
            for (int b = 0; b < 8; ++b) c = (c & 0x8000) ? (uint16_t)((c << 1) ^ 0x8005) : (uint16_t)(c << 1);
            t[i] = c;
        }
    }
};
uint16_t crc16(const uint8_t* d, size_t len) {  // x^16 + x^15 + x^2 + 1
    static const Crc16Table tab;
    uint16_t c = 0;
    for (size_t i = 0; i < len; ++i) c = (uint16_t)((c << 8) ^ tab.t[(c >> 8) ^ d[i]]);
    return c;
}

struct StreamInfo {
    int sample_rate = 0, channels = 0, bps = 0;
    int64_t total = 0;  // 0 = unknown
    int max_block = 0;
    size_t frames_at = 0;  // byte offset of the first frame
};

int parse_header(const uint8_t* d, size_t len, StreamInfo& si) {
    size_t pos = 0;
    // ID3v2 tag: "ID3", version (2), flags (1), synchsafe size (4) [+ footer]
    if (len >= 10 && memcmp(d, "ID3", 3) == 0) {
        const size_t sz = ((size_t)(d[6] & 0x7f) << 21) | ((size_t)(d[7] & 0x7f) << 14) |
                          ((size_t)(d[8] & 0x7f) << 7) | (size_t)(d[9] & 0x7f);
        pos = 10 + sz + ((d[5] & 0x10) ? 10 : 0);
    }
    AA_CHECK(pos + 4 <= len && memcmp(d + pos, "fLaC", 4) == 0, AA_ERR_INVALID, "not a FLAC stream");
    pos += 4;
    bool have_si = false, last = false;
    while (!last) {
        AA_CHECK(pos + 4 <= len, AA_ERR_INVALID, "FLAC: truncated metadata");
        last = (d[pos] & 0x80) != 0;
        const int type = d[pos] & 0x7f;
        const size_t blen = ((size_t)d[pos + 1] << 16) | ((size_t)d[pos + 2] << 8) | d[pos + 3];
        pos += 4;
        AA_CHECK(pos + blen <= len, AA_ERR_INVALID, "FLAC: truncated metadata block");
        AA_CHECK(type != 127, AA_ERR_INVALID, "FLAC: invalid metadata block type");
        if (type == 0) {
            AA_CHECK(blen >= 34 && !have_si, AA_ERR_INVALID, "FLAC: bad STREAMINFO");
            BitReader br{d + pos, blen, 0};
            br.get(16);                     // min block size
            si.max_block = (int)br.get(16); // max block size
            br.get(24);
            br.get(24);                     // min / max frame size
            si.sample_rate = (int)br.get(20);
            si.channels = (int)br.get(3) + 1;
            si.bps = (int)br.get(5) + 1;
            si.total = ((int64_t)br.get(4) << 32) | br.get(32);
            have_si = true;
        }
        pos += blen;
    }
    AA_CHECK(have_si, AA_ERR_INVALID, "FLAC: no STREAMINFO");
    AA_CHECK(si.bps >= 4, AA_ERR_INVALID, "FLAC: %d-bit samples unsupported", si.bps);
    si.frames_at = pos;
    return AA_OK;
}

// Partitioned Rice residual into res[pred_order .. block)
int read_residual(BitReader& br, int block, int pred_order, int64_t* res) {
    const int method = (int)br.get(2);
    AA_CHECK(method <= 1, AA_ERR_INVALID, "FLAC: reserved residual coding method");
    const int pbits = method == 0 ? 4 : 5, escape = method == 0 ? 15 : 31;
    const int porder = (int)br.get(4);
    const int parts = 1 << porder;
    AA_CHECK((block >> porder) << porder == block && (block >> porder) >= pred_order, AA_ERR_INVALID,
             "FLAC: bad partition order %d for block %d", porder, block);
    int i = pred_order;
    for (int p = 0; p < parts; ++p) {
        const int cnt = (block >> porder) - (p == 0 ? pred_order : 0);
        const int k = (int)br.get(pbits);
        if (k == escape) {
            const int nb = (int)br.get(5);
            for (int j = 0; j < cnt; ++j) res[i++] = br.get_signed(nb);
        } else {
            for (int j = 0; j < cnt; ++j) {
                uint32_t q;
                AA_CHECK(br.unary(q), AA_ERR_INVALID, "FLAC: truncated residual");
                const uint64_t v = ((uint64_t)q << k) | br.get(k);
                res[i++] = (int64_t)(v >> 1) ^ -(int64_t)(v & 1);
            }
        }
        AA_CHECK(!br.overrun(), AA_ERR_INVALID, "FLAC: truncated residual");
    }
    return AA_OK;
}

int read_subframe(BitReader& br, int block, int bps, int64_t* s) {
    AA_CHECK(br.get(1) == 0, AA_ERR_INVALID, "FLAC: subframe padding bit set");
    const int type = (int)br.get(6);
    int wasted = 0;
    if (br.get(1)) {
        uint32_t q;
        AA_CHECK(br.unary(q), AA_ERR_INVALID, "FLAC: truncated subframe");
        wasted = (int)q + 1;
        AA_CHECK(wasted < bps, AA_ERR_INVALID, "FLAC: %d wasted bits of %d", wasted, bps);
        bps -= wasted;
    }
    if (type == 0) {  // CONSTANT
        const int64_t v = br.get_signed(bps);
        for (int i = 0; i < block; ++i) s[i] = v;
    } else if (type == 1) {  // VERBATIM
        for (int i = 0; i < block; ++i) s[i] = br.get_signed(bps);
    } else if (type >= 8 && type <= 12) {  // FIXED, order 0-4
        const int order = type - 8;
        AA_CHECK(order <= block, AA_ERR_INVALID, "FLAC: predictor order above block size");
        for (int i = 0; i < order; ++i) s[i] = br.get_signed(bps);
        int rc = read_residual(br, block, order, s);
        if (rc) return rc;
        // predictions in wrapping uint64 arithmetic: a conforming stream never
        // overflows (identical results), a crafted one cannot reach undefined
        // behaviour
        uint64_t* u = reinterpret_cast<uint64_t*>(s);
        switch (order) {
            case 0: break;
            case 1: for (int i = 1; i < block; ++i) u[i] += u[i - 1]; break;
            case 2: for (int i = 2; i < block; ++i) u[i] += 2 * u[i - 1] - u[i - 2]; break;
            case 3: for (int i = 3; i < block; ++i) u[i] += 3 * u[i - 1] - 3 * u[i - 2] + u[i - 3]; break;
            default: for (int i = 4; i < block; ++i) u[i] += 4 * u[i - 1] - 6 * u[i - 2] + 4 * u[i - 3] - u[i - 4];
        }
    } else if (type >= 32) {  // LPC, order 1-32
        const int order = type - 31;
        AA_CHECK(order <= block, AA_ERR_INVALID, "FLAC: predictor order above block size");
        for (int i = 0; i < order; ++i) s[i] = br.get_signed(bps);
        const int prec = (int)br.get(4) + 1;
        AA_CHECK(prec != 16, AA_ERR_INVALID, "FLAC: invalid LPC precision");
        const int shift = (int)br.get_signed(5);
        AA_CHECK(shift >= 0, AA_ERR_INVALID, "FLAC: negative LPC shift");
        int64_t c[32];
        for (int j = 0; j < order; ++j) c[j] = br.get_signed(prec);
        int rc = read_residual(br, block, order, s);
        if (rc) return rc;
        for (int i = order; i < block; ++i) {  // wrapping, as above
            uint64_t acc = 0;
            for (int j = 0; j < order; ++j) acc += (uint64_t)c[j] * (uint64_t)s[i - 1 - j];
            s[i] = (int64_t)((uint64_t)s[i] + (uint64_t)((int64_t)acc >> shift));
        }
    } else {
        AA_CHECK(false, AA_ERR_INVALID, "FLAC: reserved subframe type %d", type);
    }
    AA_CHECK(!br.overrun(), AA_ERR_INVALID, "FLAC: truncated subframe");
    if (wasted)
        for (int i = 0; i < block; ++i) s[i] = (int64_t)((uint64_t)s[i] << wasted);
    return AA_OK;
}

const int kRates[12] = {0, 88200, 176400, 192000, 8000, 16000, 22050, 24000, 32000, 44100, 48000, 96000};
const int kBps[8] = {0, 8, 12, -1, 16, 20, 24, 32};

// Decode the frame at d[pos..]; on success pos moves past it.
int decode_frame(const uint8_t* d, size_t len, size_t& pos, const StreamInfo& si, std::vector<int64_t>* ch,
                 int& block, int& nch) {
    BitReader br{d, len, (uint64_t)pos * 8};
    AA_CHECK(pos + 6 <= len && br.get(15) == 0x7FFC, AA_ERR_INVALID, "FLAC: lost frame sync at byte %zu", pos);
    br.get(1);  // blocking strategy
    const int bs_code = (int)br.get(4), sr_code = (int)br.get(4);
    const int ch_code = (int)br.get(4), bps_code = (int)br.get(3);
    AA_CHECK(br.get(1) == 0 && bs_code != 0 && sr_code != 15 && ch_code <= 10 && bps_code != 3, AA_ERR_INVALID,
             "FLAC: reserved frame header value at byte %zu", pos);
    {  // coded frame / sample number: 1-7 bytes, UTF-8-like
        const uint32_t b0 = br.get(8);
        int extra = 0;
        while (extra < 8 && (b0 & (0x80u >> extra))) ++extra;
        AA_CHECK(extra != 1 && extra != 8, AA_ERR_INVALID, "FLAC: bad coded number at byte %zu", pos);
        for (int i = 1; i < extra; ++i) AA_CHECK((br.get(8) & 0xC0) == 0x80, AA_ERR_INVALID, "FLAC: bad coded number");
    }
    if (bs_code == 1) block = 192;
    else if (bs_code <= 5) block = 576 << (bs_code - 2);
    else if (bs_code == 6) block = (int)br.get(8) + 1;
    else if (bs_code == 7) block = (int)br.get(16) + 1;
    else block = 256 << (bs_code - 8);
    if (sr_code == 12) br.get(8);
    else if (sr_code == 13 || sr_code == 14) br.get(16);
    const size_t hdr_end = (size_t)(br.pos >> 3);
    AA_CHECK(hdr_end < len && crc8(d + pos, hdr_end - pos) == d[hdr_end], AA_ERR_INVALID,
             "FLAC: frame header CRC mismatch at byte %zu", pos);
    br.get(8);
    const int bps = bps_code == 0 ? si.bps : kBps[bps_code];
    AA_CHECK(bps == si.bps, AA_ERR_INVALID, "FLAC: frame bit depth %d differs from STREAMINFO's %d", bps, si.bps);
    nch = ch_code < 8 ? ch_code + 1 : 2;
    AA_CHECK(nch == si.channels, AA_ERR_INVALID, "FLAC: frame has %d channels, STREAMINFO %d", nch, si.channels);
    for (int c = 0; c < nch; ++c) {
        if ((int)ch[c].size() < block) ch[c].resize(block);
        // the side channel carries one more bit
        const bool side = (ch_code == 8 && c == 1) || (ch_code == 9 && c == 0) || (ch_code == 10 && c == 1);
        int rc = read_subframe(br, block, bps + (side ? 1 : 0), ch[c].data());
        if (rc) return rc;
    }
    br.align();
    const size_t body_end = (size_t)(br.pos >> 3);
    AA_CHECK(body_end + 2 <= len, AA_ERR_INVALID, "FLAC: truncated frame at byte %zu", pos);
    const uint16_t want = (uint16_t)((d[body_end] << 8) | d[body_end + 1]);
    AA_CHECK(crc16(d + pos, body_end - pos) == want, AA_ERR_INVALID, "FLAC: frame CRC mismatch at byte %zu", pos);
    int64_t* a = ch[0].data();
    int64_t* b = nch > 1 ? ch[1].data() : nullptr;
    // stereo decorrelation, wrapping like the predictions
    if (ch_code == 8) {         // left, side: right = left - side
        for (int i = 0; i < block; ++i) b[i] = (int64_t)((uint64_t)a[i] - (uint64_t)b[i]);
    } else if (ch_code == 9) {  // side, right: left = side + right
        for (int i = 0; i < block; ++i) a[i] = (int64_t)((uint64_t)a[i] + (uint64_t)b[i]);
    } else if (ch_code == 10) { // mid, side
        for (int i = 0; i < block; ++i) {
            const int64_t side = b[i], mid = (int64_t)((uint64_t)a[i] << 1) | (side & 1);
            a[i] = (int64_t)((uint64_t)mid + (uint64_t)side) >> 1;
            b[i] = (int64_t)((uint64_t)mid - (uint64_t)side) >> 1;
        }
    }
    pos = body_end + 2;
    return AA_OK;
}

}  // namespace

extern "C" int aa_flac_info(const uint8_t* data, size_t len, aa_flac_stream_info* info) {
    AA_CHECK(data && info, AA_ERR_INVALID, "aa_flac_info: null argument");
    StreamInfo si;
    int rc = parse_header(data, len, si);
    if (rc) return rc;
    info->sample_rate = si.sample_rate;
    info->channels = si.channels;
    info->bits_per_sample = si.bps;
    info->total_frames = si.total;
    return AA_OK;
}

extern "C" int aa_flac_decode(const uint8_t* data, size_t len, int32_t* out, int64_t cap_frames,
                              int64_t* n_frames) {
    AA_CHECK(data && n_frames && cap_frames >= 0, AA_ERR_INVALID, "aa_flac_decode: bad argument");
    StreamInfo si;
    int rc = parse_header(data, len, si);
    if (rc) return rc;
    std::vector<int64_t> ch[8];
    size_t pos = si.frames_at;
    int64_t done = 0;
    while (pos + 2 <= len && (si.total == 0 || done < si.total)) {
        if (data[pos] != 0xFF || (data[pos + 1] & 0xFE) != 0xF8) {
            // trailing bytes (e.g. an ID3v1 tag) after the last frame of a
            // stream of unknown length end the decode; anything else is damage
            AA_CHECK(si.total == 0, AA_ERR_INVALID, "FLAC: lost frame sync at byte %zu", pos);
            break;
        }
        int block = 0, nch = 0;
        rc = decode_frame(data, len, pos, si, ch, block, nch);
        if (rc) return rc;
        if (si.total) block = (int)std::min<int64_t>(block, si.total - done);
        if (out) {
            AA_CHECK(done + block <= cap_frames, AA_ERR_WORKSPACE, "aa_flac_decode: output holds %lld frames",
                     (long long)cap_frames);
            int32_t* o = out + done * nch;
            for (int i = 0; i < block; ++i)
                for (int c = 0; c < nch; ++c) o[i * nch + c] = (int32_t)ch[c][i];
        }
        done += block;
    }
    AA_CHECK(si.total == 0 || done == si.total, AA_ERR_INVALID, "FLAC: %lld of %lld samples decoded",
             (long long)done, (long long)si.total);
    *n_frames = done;
    return AA_OK;
}
