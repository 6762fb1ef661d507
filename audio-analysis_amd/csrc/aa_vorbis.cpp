// Ogg Vorbis decode on the host (C ABI aa_vorbis_*), for load_recording
// (src/identify_tracks.py:49-62), which hands every file to ffmpeg through
// audioread.  Lossy containers are the part of that path RIFF/WAVE and FLAC do
// not cover; Vorbis is the one whose decoder can be restated from its
// specification alone: every codebook, floor, residue, mapping and mode is
// transmitted in the stream's own setup header (Xiph "Vorbis I
// specification", sections 3-9), so no table has to be transcribed beyond
// floor 1's inverse-dB ramp (section 10.1, a geometric series, generated).
//
// Container: Ogg pages (RFC 3533) -- "OggS", CRC-32 (poly 0x04c11db7, the
// checksum field zeroed) verified, a damaged page skipped the way a demuxer
// resyncs; the first logical stream whose first packet is a Vorbis
// identification header is decoded, other streams are ignored.  Packets are
// reassembled from lacing values across pages.
//
// Codec: identification / comment / setup headers; codebooks (ordered and
// sparse length lists, lookup types 1 and 2); floor 0 (LSP) and floor 1;
// residue types 0, 1 and 2; mapping type 0 with submaps and square-polar
// channel coupling; short / long blocks with the window-shape transitions of
// section 4.3.1; inverse MDCT (unscaled, section 4.3.7 / 1.3.2) computed as a
// DCT-IV through an N/4-point complex FFT; overlap-add returning
// prev/4 + cur/4 samples per packet, the first audio packet none (4.3.8).
// Granule positions trim the stream: the last page's granule truncates the
// end, a first audio page whose granule is below the samples its packets
// produced drops the difference from the start (Vorbis I, A.2).
//
// Output is float32 in [-1, 1] scale, interleaved, as ffmpeg's native Vorbis
// decoder produces (AV_SAMPLE_FMT_FLTP); the caller applies libswresample's
// float -> s16 conversion and librosa's / 32768 exactly as for float WAV
// (aa_amd/audio.py).  Parity with ffmpeg's samples is unpinned: neither
// ffmpeg nor libvorbis is in the image.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "aa_common.h"

namespace {

using aa::set_error;

int ilog(uint32_t x) { return x ? 32 - __builtin_clz(x) : 0; }

// ----------------------------------------------------------------- Ogg pages
uint32_t crc_table[256];
bool crc_ready = false;

void crc_init() {
    if (crc_ready) return;
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t r = i << 24;
        for (int k = 0; k < 8; ++k) r = (r & 0x80000000u) ? (r << 1) ^ 0x04c11db7u : (r << 1);
        crc_table[i] = r;
    }
    crc_ready = true;
}

uint32_t page_crc(const uint8_t* p, size_t n) {
    uint32_t c = 0;
    for (size_t i = 0; i < n; ++i) {
        const uint8_t b = (i >= 22 && i < 26) ? 0 : p[i];  // the checksum field counts as zero
        c = (c << 8) ^ crc_table[((c >> 24) ^ b) & 0xff];
    }
    return c;
}

struct Packet {
    std::vector<uint8_t> data;
    int64_t granule = -1;   // the page granule when this is the last packet completed on its page
    int64_t page = 0;       // index of the page it completed on
};

uint32_t le32(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

// Packets of the first Vorbis logical stream, in order.  last_page: index of
// the stream's final page seen.
int read_packets(const uint8_t* d, size_t len, std::vector<Packet>& out, int64_t& last_page) {
    crc_init();
    size_t pos = 0;
    bool have_serial = false;
    uint32_t serial = 0;
    int64_t page_no = -1;
    std::vector<uint8_t> cur;
    bool in_packet = false;
    last_page = -1;
    while (pos + 27 <= len) {
        if (memcmp(d + pos, "OggS", 4) != 0) {
            ++pos;  // resync on the capture pattern
            continue;
        }
        const uint8_t* h = d + pos;
        const int nseg = h[26];
        if (h[4] != 0 || pos + 27 + nseg > len) { ++pos; continue; }
        size_t body = 0;
        for (int i = 0; i < nseg; ++i) body += h[27 + i];
        const size_t psize = 27 + nseg + body;
        if (pos + psize > len || page_crc(h, psize) != le32(h + 22)) { ++pos; continue; }
        const uint8_t type = h[5];
        int64_t granule;
        memcpy(&granule, h + 6, 8);
        const uint32_t ser = le32(h + 14);
        const uint8_t* seg = h + 27;
        const uint8_t* payload = h + 27 + nseg;
        if (!have_serial) {
            // the first beginning-of-stream page carrying a Vorbis identification header
            if ((type & 2) && nseg > 0 && body >= 7 && payload[0] == 1 && memcmp(payload + 1, "vorbis", 6) == 0) {
                have_serial = true;
                serial = ser;
            } else {
                pos += psize;
                continue;
            }
        }
        if (ser != serial) { pos += psize; continue; }
        ++page_no;
        last_page = page_no;
        if (!(type & 1) && in_packet) {  // a fresh packet starts here: the unfinished one is lost
            cur.clear();
            in_packet = false;
        }
        int j0 = 0;
        size_t o = 0;
        if ((type & 1) && !in_packet) {
            // continuation of a packet whose start was lost: skip its tail
            while (j0 < nseg) {
                o += seg[j0];
                if (seg[j0++] < 255) break;
            }
        }
        int last_done = -1;
        for (int j = j0; j < nseg; ++j) {
            cur.insert(cur.end(), payload + o, payload + o + seg[j]);
            o += seg[j];
            in_packet = true;
            if (seg[j] < 255) {
                out.push_back(Packet{std::move(cur), -1, page_no});
                cur = {};
                in_packet = false;
                last_done = (int)out.size() - 1;
            }
        }
        if (last_done >= 0) out[last_done].granule = granule;
        pos += psize;
        if (type & 4) break;  // end of stream
    }
    AA_CHECK(have_serial, AA_ERR_INVALID, "Ogg: no Vorbis stream");
    return AA_OK;
}

// ---------------------------------------------------------------- bit reader
struct Bits {
    const uint8_t* p;
    size_t n;
    uint64_t pos = 0;
    bool eop = false;
    Bits(const uint8_t* p_, size_t n_) : p(p_), n(n_) {}
    uint32_t get(int k) {  // k <= 32, LSB first (Vorbis I 2.1.4)
        if (k == 0) return 0;
        if (pos + k > (uint64_t)n * 8) {
            eop = true;
            pos = (uint64_t)n * 8;
            return 0;
        }
        const size_t b = pos >> 3;
        uint64_t v = 0;
        const size_t m = std::min<size_t>(8, n - b);
        memcpy(&v, p + b, m);
        v >>= (pos & 7);
        if (k + (pos & 7) > 64) v |= (uint64_t)p[b + 8] << (64 - (pos & 7));
        pos += k;
        return (uint32_t)(v & ((k == 32) ? 0xffffffffull : ((1ull << k) - 1)));
    }
    bool bit() { return get(1) != 0; }
};

float float32_unpack(uint32_t x) {  // Vorbis I 9.2.2
    const double mant = x & 0x1fffff;
    const int exp = (int)((x & 0x7fe00000u) >> 21);
    const double v = std::ldexp((x & 0x80000000u) ? -mant : mant, exp - 788);
    return (float)v;
}

// ------------------------------------------------------------------ codebook
struct Codebook {
    int dims = 0, entries = 0;
    std::vector<int32_t> node;   // node i: children node[2i], node[2i+1]; >0 node index, <0 leaf -(entry+1), 0 none
    int single = -1;             // the only used entry of a one-entry book
    int single_len = 0;
    int lookup = 0;
    std::vector<float> vq;       // [entries][dims] when lookup != 0

    int decode(Bits& br) const {  // entry number, -1 at end of packet / undecodable
        if (single >= 0) {
            br.get(single_len);
            return br.eop ? -1 : single;
        }
        if (node.empty()) return -1;
        int32_t at = 0;
        for (;;) {
            const int b = (int)br.get(1);
            if (br.eop) return -1;
            const int32_t nx = node[2 * at + b];
            if (nx < 0) return -nx - 1;
            if (nx == 0) return -1;
            at = nx;
        }
    }
};

// tree insertion: the leftmost free codeword of length len (Vorbis I 3.2.1)
struct TreeBuild {
    std::vector<int32_t>& node;
    std::vector<uint8_t> full;
    explicit TreeBuild(std::vector<int32_t>& n) : node(n) {
        node.assign(2, 0);
        full.assign(1, 0);
    }
    int32_t make() {
        node.push_back(0);
        node.push_back(0);
        full.push_back(0);
        return (int32_t)full.size() - 1;
    }
    bool child_full(int32_t c) const { return c < 0 || (c > 0 && full[c]); }
    // place entry at depth `left` below internal node `at`
    bool insert(int32_t at, int left, int entry) {
        if (full[at]) return false;
        for (int b = 0; b < 2; ++b) {
            int32_t c = node[2 * at + b];
            if (c < 0) continue;  // a leaf: taken
            if (left == 1) {
                if (c != 0) continue;  // an internal node: its codewords are longer
                node[2 * at + b] = -(entry + 1);
                full[at] = child_full(node[2 * at]) && child_full(node[2 * at + 1]);
                return true;
            }
            if (c == 0) {
                c = make();
                node[2 * at + b] = c;
            }
            if (insert(c, left - 1, entry)) {
                full[at] = child_full(node[2 * at]) && child_full(node[2 * at + 1]);
                return true;
            }
        }
        return false;
    }
};

int lookup1_values(int entries, int dims) {
    int r = (int)std::floor(std::pow((double)entries, 1.0 / dims));
    auto powi = [](int64_t b, int e) {
        int64_t v = 1;
        for (int i = 0; i < e; ++i) {
            v *= b;
            if (v > (int64_t)1 << 40) break;
        }
        return v;
    };
    while (r > 0 && powi(r, dims) > entries) --r;
    while (powi(r + 1, dims) <= entries) ++r;
    return r;
}

int read_codebook(Bits& br, Codebook& cb) {
    AA_CHECK(br.get(24) == 0x564342, AA_ERR_INVALID, "Vorbis: bad codebook sync");
    cb.dims = (int)br.get(16);
    cb.entries = (int)br.get(24);
    AA_CHECK(cb.dims > 0 && cb.entries > 0 && !br.eop, AA_ERR_INVALID, "Vorbis: bad codebook shape");
    std::vector<uint8_t> len(cb.entries, 0);
    if (!br.bit()) {
        const bool sparse = br.bit();
        for (int i = 0; i < cb.entries; ++i) {
            if (sparse && !br.bit()) continue;
            len[i] = (uint8_t)(br.get(5) + 1);
        }
    } else {
        int cur = 0, l = (int)br.get(5) + 1;
        while (cur < cb.entries) {
            const int num = (int)br.get(ilog((uint32_t)(cb.entries - cur)));
            AA_CHECK(cur + num <= cb.entries && l <= 32 && !br.eop, AA_ERR_INVALID, "Vorbis: bad ordered codebook");
            for (int i = 0; i < num; ++i) len[cur + i] = (uint8_t)l;
            cur += num;
            ++l;
        }
    }
    AA_CHECK(!br.eop, AA_ERR_INVALID, "Vorbis: truncated codebook");
    int used = 0, last = -1;
    for (int i = 0; i < cb.entries; ++i)
        if (len[i]) {
            ++used;
            last = i;
        }
    if (used == 1) {
        cb.single = last;
        cb.single_len = len[last];
    } else if (used > 1) {
        TreeBuild tb(cb.node);
        for (int i = 0; i < cb.entries; ++i)
            if (len[i]) AA_CHECK(tb.insert(0, len[i], i), AA_ERR_INVALID, "Vorbis: overspecified codebook");
    }
    cb.lookup = (int)br.get(4);
    AA_CHECK(cb.lookup <= 2, AA_ERR_INVALID, "Vorbis: codebook lookup type %d", cb.lookup);
    if (cb.lookup) {
        const float mn = float32_unpack(br.get(32)), delta = float32_unpack(br.get(32));
        const int vbits = (int)br.get(4) + 1;
        const bool seq = br.bit();
        const int64_t nval = cb.lookup == 1 ? lookup1_values(cb.entries, cb.dims) : (int64_t)cb.entries * cb.dims;
        AA_CHECK(nval > 0 && nval < (1 << 26), AA_ERR_INVALID, "Vorbis: bad codebook lookup size");
        std::vector<uint32_t> mult(nval);
        for (auto& m : mult) m = br.get(vbits);
        AA_CHECK(!br.eop, AA_ERR_INVALID, "Vorbis: truncated codebook lookup");
        cb.vq.resize((size_t)cb.entries * cb.dims);
        for (int e = 0; e < cb.entries; ++e) {
            float lastv = 0.f;
            int64_t div = 1;
            for (int i = 0; i < cb.dims; ++i) {
                const int64_t off = cb.lookup == 1 ? (e / div) % nval : (int64_t)e * cb.dims + i;
                const float v = (float)mult[off] * delta + mn + lastv;
                cb.vq[(size_t)e * cb.dims + i] = v;
                if (seq) lastv = v;
                if (cb.lookup == 1) div *= nval;
            }
        }
    }
    return AA_OK;
}

// -------------------------------------------------------------------- floors
struct Floor {
    int type = 1;
    // floor 0
    int order = 0, rate = 0, bark_size = 0, amp_bits = 0, amp_offset = 0;
    std::vector<int> books0;
    // floor 1
    std::vector<int> part_class;
    std::vector<int> cdim, csub, cmaster;
    std::vector<std::vector<int>> subbooks;
    int mult = 1;
    std::vector<int> X;        // X list in stream order
    std::vector<int> order1;   // indices of X sorted by value
    std::vector<int> lo, hi;   // low / high neighbours (Vorbis I 9.2.4-5)
};

int read_floor(Bits& br, Floor& f, int n_books) {
    f.type = (int)br.get(16);
    if (f.type == 0) {
        f.order = (int)br.get(8);
        f.rate = (int)br.get(16);
        f.bark_size = (int)br.get(16);
        f.amp_bits = (int)br.get(6);
        f.amp_offset = (int)br.get(8);
        const int nb = (int)br.get(4) + 1;
        for (int i = 0; i < nb; ++i) {
            f.books0.push_back((int)br.get(8));
            AA_CHECK(f.books0.back() < n_books, AA_ERR_INVALID, "Vorbis: floor 0 book out of range");
        }
        AA_CHECK(f.order > 0 && f.bark_size > 0 && f.rate > 0 && !br.eop, AA_ERR_INVALID, "Vorbis: bad floor 0");
        return AA_OK;
    }
    AA_CHECK(f.type == 1, AA_ERR_INVALID, "Vorbis: floor type %d", f.type);
    const int parts = (int)br.get(5);
    int maxc = -1;
    for (int i = 0; i < parts; ++i) {
        f.part_class.push_back((int)br.get(4));
        maxc = std::max(maxc, f.part_class.back());
    }
    f.cdim.resize(maxc + 1);
    f.csub.resize(maxc + 1);
    f.cmaster.resize(maxc + 1);
    f.subbooks.resize(maxc + 1);
    for (int c = 0; c <= maxc; ++c) {
        f.cdim[c] = (int)br.get(3) + 1;
        f.csub[c] = (int)br.get(2);
        if (f.csub[c]) {
            f.cmaster[c] = (int)br.get(8);
            AA_CHECK(f.cmaster[c] < n_books, AA_ERR_INVALID, "Vorbis: floor 1 master book out of range");
        }
        for (int j = 0; j < (1 << f.csub[c]); ++j) {
            const int b = (int)br.get(8) - 1;
            AA_CHECK(b < n_books, AA_ERR_INVALID, "Vorbis: floor 1 book out of range");
            f.subbooks[c].push_back(b);
        }
    }
    f.mult = (int)br.get(2) + 1;
    const int rb = (int)br.get(4);
    f.X = {0, 1 << rb};
    for (int i = 0; i < parts; ++i)
        for (int j = 0; j < f.cdim[f.part_class[i]]; ++j) f.X.push_back((int)br.get(rb));
    AA_CHECK(!br.eop && f.X.size() <= 65, AA_ERR_INVALID, "Vorbis: bad floor 1");
    const int nv = (int)f.X.size();
    f.order1.resize(nv);
    for (int i = 0; i < nv; ++i) f.order1[i] = i;
    std::stable_sort(f.order1.begin(), f.order1.end(), [&](int a, int b) { return f.X[a] < f.X[b]; });
    for (int i = 1; i < nv; ++i)
        AA_CHECK(f.X[f.order1[i]] != f.X[f.order1[i - 1]], AA_ERR_INVALID, "Vorbis: repeated floor 1 X");
    f.lo.assign(nv, 0);
    f.hi.assign(nv, 1);
    for (int i = 2; i < nv; ++i) {
        int lo = -1, hi = -1;
        for (int j = 0; j < i; ++j) {
            if (f.X[j] < f.X[i] && (lo < 0 || f.X[j] > f.X[lo])) lo = j;
            if (f.X[j] > f.X[i] && (hi < 0 || f.X[j] < f.X[hi])) hi = j;
        }
        f.lo[i] = lo;
        f.hi[i] = hi;
    }
    return AA_OK;
}

float inv_db[256];
bool inv_db_ready = false;

void inv_db_init() {  // Vorbis I 10.1: 1.0649863e-07 * r^i, r = 1.0649863e-07^(-1/255)
    if (inv_db_ready) return;
    for (int i = 0; i < 256; ++i) inv_db[i] = (float)std::pow(1.0649863e-07, (255.0 - i) / 255.0);
    inv_db_ready = true;
}

void render_line(int x0, int y0, int x1, int y1, float* v, int n) {  // Vorbis I 9.2.7
    const int dy = y1 - y0, adx = x1 - x0;
    int ady = std::abs(dy);
    const int base = dy / adx;
    const int sy = dy < 0 ? base - 1 : base + 1;
    ady -= std::abs(base) * adx;
    int y = y0, err = 0;
    if (x0 < n) v[x0] = inv_db[std::clamp(y, 0, 255)];
    for (int x = x0 + 1; x < x1; ++x) {
        err += ady;
        if (err >= adx) {
            err -= adx;
            y += sy;
        } else {
            y += base;
        }
        if (x < n) v[x] = inv_db[std::clamp(y, 0, 255)];
    }
}

// decode one channel's floor into curve[0..n2); false = unused
bool floor_decode(Bits& br, const Floor& f, const std::vector<Codebook>& books, int n2, float* curve,
                  std::vector<float>& scratch) {
    if (f.type == 0) {
        const uint32_t amp = br.get(f.amp_bits);
        if (br.eop || amp == 0) return false;
        const int bn = (int)br.get(ilog((uint32_t)f.books0.size()));
        if (br.eop || bn >= (int)f.books0.size()) return false;
        const Codebook& cb = books[f.books0[bn]];
        if (!cb.lookup) return false;
        std::vector<float> coef;
        float last = 0.f;
        while ((int)coef.size() < f.order) {
            const int e = cb.decode(br);
            if (e < 0) return false;
            for (int i = 0; i < cb.dims; ++i) coef.push_back(cb.vq[(size_t)e * cb.dims + i] + last);
            last = coef.back();
        }
        // curve (Vorbis I 6.2.3), f64 arithmetic
        auto bark = [](double x) { return 13.1 * std::atan(.00074 * x) + 2.24 * std::atan(.0000000185 * x * x) + .0001 * x; };
        std::vector<int> map(n2 + 1);
        const double bn2 = bark(0.5 * f.rate);
        for (int i = 0; i < n2; ++i)
            map[i] = std::min(f.bark_size - 1, (int)std::floor(bark((double)f.rate * i / (2.0 * n2)) * f.bark_size / bn2));
        map[n2] = -1;
        std::vector<double> cc(f.order);
        for (int j = 0; j < f.order; ++j) cc[j] = std::cos((double)coef[j]);
        int i = 0;
        while (i < n2) {
            const double w = M_PI * map[i] / f.bark_size, cw = std::cos(w);
            double p, q;
            if (f.order & 1) {
                p = 1.0 - cw * cw;
                for (int j = 0; j <= (f.order - 3) / 2; ++j) p *= 4.0 * (cc[2 * j + 1] - cw) * (cc[2 * j + 1] - cw);
                q = 0.25;
                for (int j = 0; j <= (f.order - 1) / 2; ++j) q *= 4.0 * (cc[2 * j] - cw) * (cc[2 * j] - cw);
            } else {
                p = (1.0 - cw) / 2.0;
                for (int j = 0; j <= (f.order - 2) / 2; ++j) p *= 4.0 * (cc[2 * j + 1] - cw) * (cc[2 * j + 1] - cw);
                q = (1.0 + cw) / 2.0;
                for (int j = 0; j <= (f.order - 2) / 2; ++j) q *= 4.0 * (cc[2 * j] - cw) * (cc[2 * j] - cw);
            }
            const double lin = std::exp(0.11512925 * ((double)amp * f.amp_offset / ((1 << f.amp_bits) - 1) /
                                                      std::sqrt(p + q) - f.amp_offset));
            const int m = map[i];
            while (i < n2 && map[i] == m) curve[i++] = (float)lin;
        }
        return true;
    }
    if (!br.bit() || br.eop) return false;
    static const int ranges[4] = {256, 128, 86, 64};
    const int range = ranges[f.mult - 1];
    const int nv = (int)f.X.size();
    int Y[65];
    const int rbits = ilog((uint32_t)(range - 1));
    Y[0] = (int)br.get(rbits);
    Y[1] = (int)br.get(rbits);
    int off = 2;
    for (size_t i = 0; i < f.part_class.size(); ++i) {
        const int c = f.part_class[i], cd = f.cdim[c], cb = f.csub[c], cs = (1 << cb) - 1;
        int cval = 0;
        if (cb) {
            cval = books[f.cmaster[c]].decode(br);
            if (cval < 0) return false;
        }
        for (int j = 0; j < cd; ++j) {
            const int book = f.subbooks[c][cval & cs];
            cval >>= cb;
            if (book >= 0) {
                const int e = books[book].decode(br);
                if (e < 0) return false;
                Y[off + j] = e;
            } else {
                Y[off + j] = 0;
            }
        }
        off += cd;
    }
    if (br.eop) return false;
    // amplitude values (Vorbis I 7.2.4 step 1)
    int fy[65];
    bool step2[65];
    fy[0] = Y[0];
    fy[1] = Y[1];
    step2[0] = step2[1] = true;
    for (int i = 2; i < nv; ++i) {
        const int lo = f.lo[i], hi = f.hi[i];
        const int x0 = f.X[lo], y0 = fy[lo], x1 = f.X[hi], y1 = fy[hi];
        const int dy = y1 - y0, adx = x1 - x0, ady = std::abs(dy);
        const int offp = ady * (f.X[i] - x0) / adx;
        const int pred = dy < 0 ? y0 - offp : y0 + offp;
        const int val = Y[i];
        const int highroom = range - pred, lowroom = pred;
        const int room = (highroom < lowroom ? highroom : lowroom) * 2;
        if (val) {
            step2[lo] = step2[hi] = true;
            step2[i] = true;
            if (val >= room)
                fy[i] = highroom > lowroom ? val - lowroom + pred : pred - val + highroom - 1;
            else
                fy[i] = (val & 1) ? pred - (val + 1) / 2 : pred + val / 2;
        } else {
            step2[i] = false;
            fy[i] = pred;
        }
    }
    // curve synthesis (step 2), in X order
    (void)scratch;
    int hx = 0, hy = 0, lx = 0, ly = fy[f.order1[0]] * f.mult;
    for (int k = 1; k < nv; ++k) {
        const int i = f.order1[k];
        if (step2[i]) {
            hy = fy[i] * f.mult;
            hx = f.X[i];
            render_line(lx, ly, hx, hy, curve, n2);
            lx = hx;
            ly = hy;
        }
    }
    if (hx < n2) render_line(hx, hy, n2, hy, curve, n2);
    return true;
}

// ------------------------------------------------------------------ residues
struct Residue {
    int type = 0, begin = 0, end = 0, psize = 1, classes = 1, classbook = 0;
    std::vector<int> books;  // [classes][8], -1 = none
};

int read_residue(Bits& br, Residue& r, const std::vector<Codebook>& books) {
    r.type = (int)br.get(16);
    AA_CHECK(r.type <= 2, AA_ERR_INVALID, "Vorbis: residue type %d", r.type);
    r.begin = (int)br.get(24);
    r.end = (int)br.get(24);
    r.psize = (int)br.get(24) + 1;
    r.classes = (int)br.get(6) + 1;
    r.classbook = (int)br.get(8);
    AA_CHECK(r.classbook < (int)books.size() && !br.eop, AA_ERR_INVALID, "Vorbis: bad residue header");
    std::vector<int> casc(r.classes);
    for (int c = 0; c < r.classes; ++c) {
        int low = (int)br.get(3), high = 0;
        if (br.bit()) high = (int)br.get(5);
        casc[c] = high * 8 + low;
    }
    r.books.assign(r.classes * 8, -1);
    for (int c = 0; c < r.classes; ++c)
        for (int p = 0; p < 8; ++p)
            if (casc[c] & (1 << p)) {
                const int b = (int)br.get(8);
                AA_CHECK(b < (int)books.size() && books[b].lookup, AA_ERR_INVALID, "Vorbis: bad residue book");
                r.books[c * 8 + p] = b;
            }
    AA_CHECK(!br.eop, AA_ERR_INVALID, "Vorbis: truncated residue header");
    return AA_OK;
}

// residue formats 0 / 1 over vectors v[ch] of length n (Vorbis I 8.6.2-4)
void residue_decode01(Bits& br, const Residue& r, const std::vector<Codebook>& books, int type,
                      std::vector<float*>& v, const std::vector<bool>& dnd, int n) {
    const int ch = (int)v.size();
    const int lb = std::min(r.begin, n), le = std::min(r.end, n);
    const int ntr = le - lb;
    if (ntr <= 0) return;
    const int nparts = ntr / r.psize;
    const Codebook& cbk = books[r.classbook];
    const int cpw = cbk.dims;
    std::vector<int> cls((size_t)ch * (nparts + cpw), 0);
    for (int pass = 0; pass < 8; ++pass) {
        int pc = 0;
        while (pc < nparts) {
            if (pass == 0) {
                for (int j = 0; j < ch; ++j) {
                    if (dnd[j]) continue;
                    int temp = cbk.decode(br);
                    if (temp < 0) return;
                    for (int i = cpw - 1; i >= 0; --i) {
                        cls[(size_t)j * (nparts + cpw) + i + pc] = temp % r.classes;
                        temp /= r.classes;
                    }
                }
            }
            for (int i = 0; i < cpw && pc < nparts; ++i, ++pc) {
                for (int j = 0; j < ch; ++j) {
                    if (dnd[j]) continue;
                    const int c = cls[(size_t)j * (nparts + cpw) + pc];
                    const int bk = r.books[c * 8 + pass];
                    if (bk < 0) continue;
                    const Codebook& cb = books[bk];
                    float* out = v[j] + lb + pc * r.psize;
                    if (type == 0) {
                        const int step = r.psize / cb.dims;
                        for (int s = 0; s < step; ++s) {
                            const int e = cb.decode(br);
                            if (e < 0) return;
                            const float* vec = &cb.vq[(size_t)e * cb.dims];
                            for (int k = 0; k < cb.dims; ++k) out[s + k * step] += vec[k];
                        }
                    } else {
                        int s = 0;
                        while (s < r.psize) {
                            const int e = cb.decode(br);
                            if (e < 0) return;
                            const float* vec = &cb.vq[(size_t)e * cb.dims];
                            for (int k = 0; k < cb.dims && s < r.psize; ++k) out[s++] += vec[k];
                        }
                    }
                }
            }
        }
    }
}

// --------------------------------------------------------------------- IMDCT
// y[n] = sum_k X[k] cos(2 pi / N (n + 1/2 + N/4)(k + 1/2)), n < N, k < N/2:
// u = DCT-IV of size M = N/2 (pre-twiddle, M/2-point complex FFT,
// post-twiddle), then y[n] = u[n + M/2] for n < M/2, -u[3M/2 - 1 - n] for
// n < 3M/2, -u[n - 3M/2] above.
struct Imdct {
    int N = 0;
    std::vector<double> tw_pre_c, tw_pre_s, tw_post_c, tw_post_s, fft_c, fft_s;
    std::vector<int> rev;
    void init(int n) {
        N = n;
        const int M = N / 2, Q = M / 2;
        tw_pre_c.resize(Q);
        tw_pre_s.resize(Q);
        tw_post_c.resize(Q);
        tw_post_s.resize(Q);
        for (int k = 0; k < Q; ++k) {
            tw_pre_c[k] = std::cos(-M_PI * (k + 0.25) / M);
            tw_pre_s[k] = std::sin(-M_PI * (k + 0.25) / M);
            tw_post_c[k] = std::cos(-M_PI * k / M);
            tw_post_s[k] = std::sin(-M_PI * k / M);
        }
        fft_c.resize(Q / 2 + 1);
        fft_s.resize(Q / 2 + 1);
        for (int k = 0; k <= Q / 2; ++k) {
            fft_c[k] = std::cos(-2.0 * M_PI * k / Q);
            fft_s[k] = std::sin(-2.0 * M_PI * k / Q);
        }
        rev.resize(Q);
        const int bits = ilog((uint32_t)Q) - 1;
        for (int i = 0; i < Q; ++i) {
            int r = 0;
            for (int b = 0; b < bits; ++b)
                if (i & (1 << b)) r |= 1 << (bits - 1 - b);
            rev[i] = r;
        }
    }
    void run(const float* X, float* y, std::vector<double>& re, std::vector<double>& im) const {
        const int M = N / 2, Q = M / 2;
        re.resize(Q);
        im.resize(Q);
        for (int k = 0; k < Q; ++k) {
            const double a = X[2 * k], b = X[M - 1 - 2 * k];
            const int r = rev[k];
            re[r] = a * tw_pre_c[k] - b * tw_pre_s[k];
            im[r] = a * tw_pre_s[k] + b * tw_pre_c[k];
        }
        for (int len = 2; len <= Q; len <<= 1) {
            const int half = len / 2, step = Q / len;
            for (int s = 0; s < Q; s += len)
                for (int j = 0; j < half; ++j) {
                    const double wc = fft_c[j * step], ws = fft_s[j * step];
                    const int a = s + j, b = a + half;
                    const double tr = re[b] * wc - im[b] * ws, ti = re[b] * ws + im[b] * wc;
                    re[b] = re[a] - tr;
                    im[b] = im[a] - ti;
                    re[a] += tr;
                    im[a] += ti;
                }
        }
        // u[2k] = Re(c_k), u[M-1-2k] = -Im(c_k), c = V * post twiddle
        auto u = [&](int m) -> double {
            const int k = (m & 1) ? (M - 1 - m) / 2 : m / 2;
            const double cr = re[k] * tw_post_c[k] - im[k] * tw_post_s[k];
            const double ci = re[k] * tw_post_s[k] + im[k] * tw_post_c[k];
            return (m & 1) ? -ci : cr;
        };
        for (int n = 0; n < M / 2; ++n) y[n] = (float)u(n + M / 2);
        for (int n = M / 2; n < 3 * M / 2; ++n) y[n] = (float)-u(3 * M / 2 - 1 - n);
        for (int n = 3 * M / 2; n < N; ++n) y[n] = (float)-u(n - 3 * M / 2);
    }
};

// ------------------------------------------------------------------- decoder
struct Mapping {
    int submaps = 1;
    std::vector<int> mag, ang, mux, sub_floor, sub_res;
};
struct Mode {
    int blockflag = 0, mapping = 0;
};

struct Decoder {
    int channels = 0, rate = 0, bs[2] = {0, 0};
    std::vector<Codebook> books;
    std::vector<Floor> floors;
    std::vector<Residue> residues;
    std::vector<Mapping> maps;
    std::vector<Mode> modes;
    Imdct mdct[2];
    std::vector<float> win[2][2][2];  // [blockflag][prev long][next long]

    int ident(const Packet& p) {
        Bits br(p.data.data(), p.data.size());
        AA_CHECK(p.data.size() >= 30 && p.data[0] == 1 && memcmp(&p.data[1], "vorbis", 6) == 0, AA_ERR_INVALID,
                 "Vorbis: bad identification header");
        br.pos = 7 * 8;
        AA_CHECK(br.get(32) == 0, AA_ERR_INVALID, "Vorbis: unsupported version");
        channels = (int)br.get(8);
        rate = (int)br.get(32);
        br.get(32);
        br.get(32);
        br.get(32);
        bs[0] = 1 << br.get(4);
        bs[1] = 1 << br.get(4);
        const bool framing = br.bit();
        AA_CHECK(channels > 0 && rate > 0 && bs[0] >= 64 && bs[1] <= 8192 && bs[0] <= bs[1] && framing,
                 AA_ERR_INVALID, "Vorbis: bad identification header fields");
        return AA_OK;
    }

    int setup(const Packet& p) {
        AA_CHECK(p.data.size() >= 7 && p.data[0] == 5 && memcmp(&p.data[1], "vorbis", 6) == 0, AA_ERR_INVALID,
                 "Vorbis: bad setup header");
        Bits br(p.data.data(), p.data.size());
        br.pos = 7 * 8;
        const int nb = (int)br.get(8) + 1;
        books.resize(nb);
        for (auto& b : books) {
            int rc = read_codebook(br, b);
            if (rc) return rc;
        }
        const int nt = (int)br.get(6) + 1;
        for (int i = 0; i < nt; ++i) AA_CHECK(br.get(16) == 0, AA_ERR_INVALID, "Vorbis: bad time-domain transform");
        floors.resize(br.get(6) + 1);
        for (auto& f : floors) {
            int rc = read_floor(br, f, nb);
            if (rc) return rc;
        }
        residues.resize(br.get(6) + 1);
        for (auto& r : residues) {
            int rc = read_residue(br, r, books);
            if (rc) return rc;
        }
        maps.resize(br.get(6) + 1);
        for (auto& m : maps) {
            AA_CHECK(br.get(16) == 0, AA_ERR_INVALID, "Vorbis: mapping type");
            m.submaps = br.bit() ? (int)br.get(4) + 1 : 1;
            if (br.bit()) {
                const int steps = (int)br.get(8) + 1;
                const int bits = ilog((uint32_t)(channels - 1));
                for (int s = 0; s < steps; ++s) {
                    const int a = (int)br.get(bits), b = (int)br.get(bits);
                    AA_CHECK(a != b && a < channels && b < channels, AA_ERR_INVALID, "Vorbis: bad coupling step");
                    m.mag.push_back(a);
                    m.ang.push_back(b);
                }
            }
            AA_CHECK(br.get(2) == 0, AA_ERR_INVALID, "Vorbis: mapping reserved bits");
            m.mux.assign(channels, 0);
            if (m.submaps > 1)
                for (auto& x : m.mux) {
                    x = (int)br.get(4);
                    AA_CHECK(x < m.submaps, AA_ERR_INVALID, "Vorbis: bad mapping mux");
                }
            for (int s = 0; s < m.submaps; ++s) {
                br.get(8);
                m.sub_floor.push_back((int)br.get(8));
                m.sub_res.push_back((int)br.get(8));
                AA_CHECK(m.sub_floor.back() < (int)floors.size() && m.sub_res.back() < (int)residues.size(),
                         AA_ERR_INVALID, "Vorbis: mapping submap out of range");
            }
        }
        modes.resize(br.get(6) + 1);
        for (auto& md : modes) {
            md.blockflag = (int)br.get(1);
            AA_CHECK(br.get(16) == 0 && br.get(16) == 0, AA_ERR_INVALID, "Vorbis: mode window / transform type");
            md.mapping = (int)br.get(8);
            AA_CHECK(md.mapping < (int)maps.size(), AA_ERR_INVALID, "Vorbis: mode mapping out of range");
        }
        AA_CHECK(br.bit() && !br.eop, AA_ERR_INVALID, "Vorbis: setup header framing");
        for (int f = 0; f < 2; ++f) mdct[f].init(bs[f]);
        for (int f = 0; f < 2; ++f)
            for (int pl = 0; pl < 2; ++pl)
                for (int nl = 0; nl < 2; ++nl) make_window(win[f][pl][nl], f, pl, nl);
        inv_db_init();
        return AA_OK;
    }

    void make_window(std::vector<float>& w, int f, int prev_long, int next_long) const {  // Vorbis I 4.3.1
        const int n = bs[f];
        w.assign(n, 0.f);
        int ls, le, ln, rs, re, rn;
        if (f && !prev_long) {
            ls = n / 4 - bs[0] / 4; le = n / 4 + bs[0] / 4; ln = bs[0] / 2;
        } else {
            ls = 0; le = n / 2; ln = n / 2;
        }
        if (f && !next_long) {
            rs = n * 3 / 4 - bs[0] / 4; re = n * 3 / 4 + bs[0] / 4; rn = bs[0] / 2;
        } else {
            rs = n / 2; re = n; rn = n / 2;
        }
        for (int i = ls; i < le; ++i) {
            const double s = std::sin((i - ls + 0.5) / ln * M_PI / 2);
            w[i] = (float)std::sin(M_PI / 2 * s * s);
        }
        for (int i = le; i < rs; ++i) w[i] = 1.f;
        for (int i = rs; i < re; ++i) {
            const double s = std::sin((i - rs + 0.5) / rn * M_PI / 2 + M_PI / 2);
            w[i] = (float)std::sin(M_PI / 2 * s * s);
        }
    }

    // one audio packet -> windowed block (n samples per channel) in blk;
    // returns n, 0 to skip the packet
    int audio(const Packet& p, std::vector<std::vector<float>>& blk, int& lstart, int& rend,
              std::vector<std::vector<float>>& res, std::vector<float>& curve, std::vector<double>& re,
              std::vector<double>& im) {
        Bits br(p.data.data(), p.data.size());
        if (p.data.empty() || br.get(1) != 0) return 0;
        const int mn = (int)br.get(ilog((uint32_t)(modes.size() - 1)));
        if (br.eop || mn >= (int)modes.size()) return 0;
        const Mode& md = modes[mn];
        const int f = md.blockflag, n = bs[f], n2 = n / 2;
        int pl = 1, nl = 1;
        if (f) {
            pl = (int)br.get(1);
            nl = (int)br.get(1);
        }
        const auto& w = win[f][f ? pl : 1][f ? nl : 1];
        const Mapping& m = maps[md.mapping];
        res.resize(channels);
        std::vector<bool> nz(channels, false);
        std::vector<std::vector<float>> floorc(channels);
        for (int c = 0; c < channels; ++c) {
            res[c].assign(n2, 0.f);
            floorc[c].assign(n2, 0.f);
            const Floor& fl = floors[m.sub_floor[m.mux[c]]];
            nz[c] = floor_decode(br, fl, books, n2, floorc[c].data(), curve);
        }
        std::vector<bool> no_res(channels);
        for (int c = 0; c < channels; ++c) no_res[c] = !nz[c];
        for (size_t s = 0; s < m.mag.size(); ++s)
            if (!no_res[m.mag[s]] || !no_res[m.ang[s]]) no_res[m.mag[s]] = no_res[m.ang[s]] = false;
        for (int s = 0; s < m.submaps; ++s) {
            std::vector<int> chs;
            for (int c = 0; c < channels; ++c)
                if (m.mux[c] == s) chs.push_back(c);
            const Residue& r = residues[m.sub_res[s]];
            std::vector<bool> dnd;
            for (int c : chs) dnd.push_back(no_res[c]);
            if (r.type == 2) {
                bool any = false;
                for (bool d : dnd) any |= !d;
                if (!any) continue;
                const int k = (int)chs.size();
                std::vector<float> tmp((size_t)n2 * k, 0.f);
                std::vector<float*> v{tmp.data()};
                residue_decode01(br, r, books, 1, v, std::vector<bool>{false}, n2 * k);
                for (int j = 0; j < n2; ++j)
                    for (int i = 0; i < k; ++i) res[chs[i]][j] = tmp[(size_t)j * k + i];
            } else {
                std::vector<float*> v;
                for (int c : chs) v.push_back(res[c].data());
                residue_decode01(br, r, books, r.type, v, dnd, n2);
            }
        }
        for (int s = (int)m.mag.size() - 1; s >= 0; --s) {  // inverse coupling (Vorbis I 4.3.5)
            float* M_ = res[m.mag[s]].data();
            float* A = res[m.ang[s]].data();
            for (int j = 0; j < n2; ++j) {
                const float M0 = M_[j], A0 = A[j];
                float nm, na;
                if (M0 > 0) {
                    if (A0 > 0) { nm = M0; na = M0 - A0; } else { na = M0; nm = M0 + A0; }
                } else {
                    if (A0 > 0) { nm = M0; na = M0 + A0; } else { na = M0; nm = M0 - A0; }
                }
                M_[j] = nm;
                A[j] = na;
            }
        }
        blk.resize(channels);
        for (int c = 0; c < channels; ++c) {
            blk[c].assign(n, 0.f);
            if (!nz[c]) continue;  // unused floor: the channel is silent
            for (int j = 0; j < n2; ++j) res[c][j] *= floorc[c][j];
            mdct[f].run(res[c].data(), blk[c].data(), re, im);
            for (int i = 0; i < n; ++i) blk[c][i] *= w[i];
        }
        // the window's nonzero span
        lstart = 0;
        rend = n;
        if (f && !pl) lstart = n / 4 - bs[0] / 4;
        if (f && !nl) rend = n * 3 / 4 + bs[0] / 4;
        return n;
    }
};

struct Decoded {
    int channels = 0, rate = 0, bs0 = 0, bs1 = 0;
    int64_t total = 0;   // samples per channel after trimming
};

// decode the whole stream; out (interleaved) when non-null
int decode_all(const uint8_t* data, size_t len, float* out, int64_t cap, Decoded& dec, bool headers_only) {
    std::vector<Packet> pk;
    int64_t last_page = -1;
    int rc = read_packets(data, len, pk, last_page);
    if (rc) return rc;
    AA_CHECK(pk.size() >= 3, AA_ERR_INVALID, "Vorbis: missing headers");
    Decoder D;
    rc = D.ident(pk[0]);
    if (rc) return rc;
    AA_CHECK(pk[1].data.size() >= 7 && pk[1].data[0] == 3 && memcmp(&pk[1].data[1], "vorbis", 6) == 0,
             AA_ERR_INVALID, "Vorbis: bad comment header");
    rc = D.setup(pk[2]);
    if (rc) return rc;
    dec.channels = D.channels;
    dec.rate = D.rate;
    dec.bs0 = D.bs[0];
    dec.bs1 = D.bs[1];
    if (headers_only) {
        int64_t g = -1;
        for (size_t i = 3; i < pk.size(); ++i)
            if (pk[i].granule >= 0) g = pk[i].granule;
        dec.total = std::max<int64_t>(g, 0);
        return AA_OK;
    }
    const int C = D.channels;
    // timeline of windowed blocks: block k starts at pk_pos (p_0 = bs1)
    std::vector<std::vector<float>> acc(C);
    std::vector<std::vector<float>> blk, res;
    std::vector<float> curve;
    std::vector<double> re, im;
    int64_t p = D.bs[1], prev_n = 0, prev_center = -1, first_center = -1;
    int64_t produced = 0;             // samples final so far (from the first block's centre)
    int64_t start_trim = 0, end_total = -1;
    bool first_granule_seen = false;
    for (size_t i = 3; i < pk.size(); ++i) {
        int ls = 0, rend = 0;
        const int n = D.audio(pk[i], blk, ls, rend, res, curve, re, im);
        if (n > 0) {
            if (prev_n) p += 3 * prev_n / 4 - n / 4;
            const int64_t need = p + n;
            for (int c = 0; c < C; ++c) {
                if ((int64_t)acc[c].size() < need) acc[c].resize(std::max<int64_t>(need, (int64_t)acc[c].size() * 2), 0.f);
                float* a = acc[c].data() + p;
                for (int s = ls; s < rend; ++s) a[s] += blk[c][s];
            }
            const int64_t center = p + n / 2;
            if (prev_center < 0) first_center = center;
            else produced += center - prev_center;
            prev_center = center;
            prev_n = n;
        }
        if (pk[i].granule >= 0) {
            const bool last = pk[i].page == last_page;
            if (!first_granule_seen && !last && pk[i].granule < produced) start_trim = produced - pk[i].granule;
            first_granule_seen = true;
            if (last) end_total = pk[i].granule;
        }
    }
    int64_t total = produced - start_trim;
    if (end_total >= 0) total = std::min(total, end_total);
    total = std::max<int64_t>(total, 0);
    dec.total = total;
    if (out) {
        AA_CHECK(total <= cap, AA_ERR_WORKSPACE, "aa_vorbis_decode: output holds %lld frames", (long long)cap);
        const int64_t s0 = first_center + start_trim;
        for (int64_t t = 0; t < total; ++t)
            for (int c = 0; c < C; ++c) out[t * C + c] = acc[c][s0 + t];
    }
    return AA_OK;
}

}  // namespace

extern "C" int aa_vorbis_info(const uint8_t* data, size_t len, aa_vorbis_stream_info* info) {
    AA_CHECK(data && info, AA_ERR_INVALID, "aa_vorbis_info: null argument");
    Decoded d;
    int rc = decode_all(data, len, nullptr, 0, d, true);
    if (rc) return rc;
    info->sample_rate = d.rate;
    info->channels = d.channels;
    info->blocksize_0 = d.bs0;
    info->blocksize_1 = d.bs1;
    info->total_frames = d.total;
    return AA_OK;
}

extern "C" int aa_vorbis_decode(const uint8_t* data, size_t len, float* out, int64_t cap_frames,
                                int64_t* n_frames) {
    AA_CHECK(data && n_frames && cap_frames >= 0, AA_ERR_INVALID, "aa_vorbis_decode: bad argument");
    Decoded d;
    int rc = decode_all(data, len, out, cap_frames, d, false);
    if (rc) return rc;
    *n_frames = d.total;
    return AA_OK;
}
