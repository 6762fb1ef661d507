// Track builder on the host (C ABI aa_tracks_from_signals): the merge sweeps
// and the enlarge / absorb / narrow-drop pass of get_tracks_from_signals
// (src/identify_tracks.py:725-842, restated in aa_amd/identify_tracks.py),
// for the batched corpus path (aa_amd/batch.py), whose lane threads otherwise
// spend a large share of their interpreter time in that Python loop nest
// (~84 segment overlaps per file) while the GIL serialises them.
//
// The arithmetic is Python's, step for step, in IEEE double (SSE2; no
// contraction): the same operand order, min / max returning their first
// argument on ties, int() as truncation.  Python's int / float distinction of
// a field survives the arithmetic only through min / max, enlarge's int()
// and max(start - pad, 0), and it shows in the JSON (0 against 0.0), so every
// field carries it.  Mel values are never recomputed here: a signal's come
// with it (numpy's log10 is not libm's to the last bit), a merge keeps the
// mel of the frequency it keeps, and enlarge's integer frequencies look
// theirs up in a table the caller built with numpy (the same values as
// aa_amd.identify_tracks.mel_freq).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "aa_common.h"

#pragma clang fp contract(off)

namespace {

struct Num {
    double v;
    bool i;  // a Python int
};

struct Sig {
    Num start, end, fs, fe;
    double ms, me;  // mel of fs / fe
    bool del;
};

// Python's min(a, b) / max(a, b): the first argument unless the second is
// strictly smaller / larger
inline Num pymin(const Num& a, const Num& b) { return b.v < a.v ? b : a; }
inline Num pymax(const Num& a, const Num& b) { return b.v > a.v ? b : a; }
inline double dmax(double a, double b) { return b > a ? b : a; }
inline double dmin(double a, double b) { return b < a ? b : a; }

// segment_overlap (:709-710)
inline double seg(double a0, double a1, double b0, double b1) {
    return (a1 - a0) + (b1 - b0) - (dmax(a1, b1) - dmin(a0, b0));
}

inline double len(const Sig& s) { return s.end.v - s.start.v; }
inline double mel_range(const Sig& s) { return s.me - s.ms; }

// Signal.merge: the extremes of both, each frequency with its own mel
inline void merge(Sig& s, const Sig& u) {
    s.start = pymin(s.start, u.start);
    s.end = pymax(s.end, u.end);
    if (u.fs.v < s.fs.v) {
        s.fs = u.fs;
        s.ms = u.ms;
    }
    if (u.fe.v > s.fe.v) {
        s.fe = u.fe;
        s.me = u.me;
    }
}

enum { OK = 0, ZERO_DIV = 1, MEL_RANGE = 2 };

// merge_signals (:725-792) over the live signals `live` (indices into sig):
// the new live list in the sweep's order; *merged if any merge happened
int merge_sweep(std::vector<Sig>& sig, std::vector<int>& live, bool* merged_any) {
    // sorted by mel_freq_end descending, then (stable) by start
    std::stable_sort(live.begin(), live.end(), [&](int a, int b) { return sig[a].me > sig[b].me; });
    std::stable_sort(live.begin(), live.end(), [&](int a, int b) { return sig[a].start.v < sig[b].start.v; });
    *merged_any = false;
    for (int si : live) {
        Sig& s = sig[si];
        if (s.del) continue;
        int absorbed = -1;
        for (int ui : live) {
            const Sig& u = sig[ui];
            if (u.del || ui == si) continue;
            const bool same_side = (u.me < 1500 && s.me < 1500) || (u.me > 1500 && s.me > 1500);
            if (!same_side) continue;
            const double overlap = seg(s.start.v, s.end.v, u.start.v, u.end.v);
            const double fot = (s.ms > 1000 && u.ms > 1000) ? 0.5 : 0.75;
            const double time_diff = s.start.v > u.end.v ? s.start.v - u.end.v : u.start.v - s.end.v;
            const double mel_overlap = seg(s.ms, s.me, u.ms, u.me);
            if (overlap > len(u) * 0.75 && mel_overlap > -20) {
                absorbed = ui;
            } else if (overlap > 0 && mel_overlap > mel_range(u) * fot) {
                absorbed = ui;
            } else if (mel_overlap > mel_range(u) * fot && time_diff <= 2) {
                // (sic) u's mel end against s's mel range, as the reference
                double range_overlap;
                if (u.me > mel_range(s)) {
                    if (mel_range(u) == 0) return ZERO_DIV;
                    range_overlap = mel_range(s) / mel_range(u);
                } else {
                    if (mel_range(s) == 0) return ZERO_DIV;
                    range_overlap = mel_range(u) / mel_range(s);
                }
                if (range_overlap < 0.75) continue;
                absorbed = ui;
            }
            if (absorbed >= 0) {
                merge(s, u);
                break;
            }
        }
        if (absorbed >= 0) {
            *merged_any = true;
            sig[absorbed].del = true;
        }
    }
    live.erase(std::remove_if(live.begin(), live.end(), [&](int i) { return sig[i].del; }), live.end());
    return OK;
}

// Signal.enlarge(scale, min_track_length)
int enlarge(Sig& s, double scale, double min_track_length, const double* mel_int, int64_t n_mel) {
    const double length = len(s);
    const double grown = dmax(length * scale, min_track_length);
    const double pad = (grown - length) / 2;
    const double st = s.start.v - pad;
    s.start = 0 > st ? Num{0.0, true} : Num{st, false};
    s.end = Num{s.end.v + pad, false};
    const double fpad = ((s.fe.v - s.fs.v) * scale - (s.fe.v - s.fs.v)) / 2;
    const double lo = s.fs.v - fpad;
    const double fe = std::trunc(s.fe.v + fpad);
    const double fs = std::trunc(0 > lo ? 0.0 : lo);
    if (!(fe >= 0 && fe < (double)n_mel && fs >= 0 && fs < (double)n_mel)) return MEL_RANGE;
    s.fe = Num{fe + 0.0, true};  // int(-0.0) is 0
    s.fs = Num{fs + 0.0, true};
    s.me = mel_int[(int64_t)fe];
    s.ms = mel_int[(int64_t)fs];
    return OK;
}

}  // namespace

extern "C" int aa_tracks_from_signals(const double* sig_in, const int32_t* kind_in, int64_t n, double end,
                                      int32_t end_is_int, const double* mel_int, int64_t n_mel, double* track_out,
                                      int32_t* kind_out, int64_t* n_tracks) {
    AA_CHECK(n >= 0 && n_tracks && (n == 0 || (sig_in && kind_in && track_out && kind_out)) && mel_int && n_mel > 0,
             AA_ERR_INVALID, "aa_tracks_from_signals: bad arguments");
    *n_tracks = 0;
    // NaN keys would break the sorts' strict weak order (Python's sort copes):
    // such inputs stay with the Python builder
    bool nan = std::isnan(end);
    for (int64_t k = 0; k < 6 * n; ++k) nan = nan || std::isnan(sig_in[k]);
    if (nan) {
        aa::set_error("aa_tracks_from_signals: NaN in the signals or the end");
        return AA_ERR_UNSUPPORTED;
    }
    std::vector<Sig> sig((size_t)n);
    std::vector<int> live((size_t)n);
    for (int64_t k = 0; k < n; ++k) {
        const double* r = sig_in + 6 * k;
        const int32_t f = kind_in[k];
        sig[k] = Sig{{r[0], (f & 1) != 0}, {r[1], (f & 2) != 0}, {r[2], (f & 4) != 0}, {r[3], (f & 8) != 0},
                     r[4], r[5], false};
        live[k] = (int)k;
    }
    // get_tracks_from_signals (:795-842)
    bool merged = true;
    while (merged) {
        if (merge_sweep(sig, live, &merged) != OK) {
            aa::set_error("aa_tracks_from_signals: zero mel range in a merge test (Python raises here)");
            return AA_ERR_INVALID;
        }
    }
    double min_length = 0.35;
    const double min_track_length = 0.7;
    const Num endn{end, end_is_int != 0};
    for (int si : live) {
        Sig& s = sig[si];
        if (s.del) continue;
        if (len(s) < min_length) {
            s.del = true;
            continue;
        }
        if (enlarge(s, 1.4, min_track_length, mel_int, n_mel) != OK) {
            aa::set_error("aa_tracks_from_signals: enlarged frequency outside the %lld-entry mel table",
                          (long long)n_mel);
            return AA_ERR_UNSUPPORTED;
        }
        s.end = pymin(endn, s.end);
        for (int s2i : live) {
            Sig& s2 = sig[s2i];
            if (s2.del || s2i == si) continue;
            const double overlap = seg(s.start.v, s.end.v, s2.start.v, s2.end.v);
            min_length = dmin(len(s), len(s2));
            if (overlap > 0.7 * min_length) {
                merge(s, s2);
                s2.del = true;
            }
        }
    }
    int64_t m = 0;
    for (int si : live) {
        const Sig& s = sig[si];
        if (s.del || mel_range(s) < 50) continue;
        double* o = track_out + 6 * m;
        o[0] = s.start.v;
        o[1] = s.end.v;
        o[2] = s.fs.v;
        o[3] = s.fe.v;
        o[4] = s.ms;
        o[5] = s.me;
        kind_out[m] = (s.start.i ? 1 : 0) | (s.end.i ? 2 : 0) | (s.fs.i ? 4 : 0) | (s.fe.i ? 8 : 0);
        ++m;
    }
    *n_tracks = m;
    return AA_OK;
}
