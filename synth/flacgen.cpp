// flacgen.cpp -- seeded synthetic FLAC writer. See flacgen.h.
//
// Format written per RFC 9639; choices that matter for zflac parity:
//  * side channels use CONSTANT subframes only on request (`const_side`): zflac reads
//    `bits_per_sample` bits for them (src/zflac.zig:447), the RFC reads bps+1; both widths
//    can be written so the quirk and its mismatch with RFC encoders are testable;
//  * side channels fit the SampleType container (src/zflac.zig:494,537,558,564) unless
//    `allow_side_overflow` asks for an out-of-domain stream;
//  * every LPC partial sum is checked against the InterType width in the order zflac
//    accumulates it (src/zflac.zig:527-532), so Debug zflac would not trap;
//  * the block size is always divisible by 2^partition_order (src/zflac.zig:623-632).
#include "flacgen.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../zflac_amd/csrc/md5.hpp"

namespace {

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x1234567ull) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
    double gauss() {  // Irwin-Hall(4) scaled to unit variance: cheap and bounded
        double a = uniform() + uniform() + uniform() + uniform() - 2.0;
        return a * 1.7320508075688772;
    }
};

class BitWriter {
public:
    std::vector<uint8_t> buf;
    void put(uint64_t v, int bits) {
        while (bits > 0) {
            int take = bits > 32 ? 32 : bits;
            uint64_t chunk = (v >> (bits - take)) & ((take == 64) ? ~0ull : ((1ull << take) - 1));
            acc_ = (acc_ << take) | chunk;
            n_ += take;
            bits -= take;
            while (n_ >= 8) {
                buf.push_back(static_cast<uint8_t>(acc_ >> (n_ - 8)));
                n_ -= 8;
            }
            acc_ &= (1ull << n_) - 1;
        }
    }
    void put_signed(int64_t v, int bits) { put(static_cast<uint64_t>(v) & ((bits == 64) ? ~0ull : ((1ull << bits) - 1)), bits); }
    void unary(uint64_t q) {
        while (q >= 32) {
            put(0, 32);
            q -= 32;
        }
        put(1, static_cast<int>(q) + 1);
    }
    void align() {
        if (n_) put(0, 8 - n_);
    }
    size_t bytes() const { return buf.size(); }

private:
    uint64_t acc_ = 0;
    int n_ = 0;
};

uint8_t crc8(const uint8_t* p, size_t n) {
    uint8_t c = 0;
    for (size_t i = 0; i < n; i++) {
        c ^= p[i];
        for (int b = 0; b < 8; b++) c = static_cast<uint8_t>((c & 0x80) ? (c << 1) ^ 0x07 : (c << 1));
    }
    return c;
}
uint16_t crc16(const uint8_t* p, size_t n) {
    uint16_t c = 0;
    for (size_t i = 0; i < n; i++) {
        c ^= static_cast<uint16_t>(p[i] << 8);
        for (int b = 0; b < 8; b++) c = static_cast<uint16_t>((c & 0x8000) ? (c << 1) ^ 0x8005 : (c << 1));
    }
    return c;
}

inline bool fits(int64_t v, int bits) {
    if (bits >= 64) return true;
    const int64_t lo = -(int64_t(1) << (bits - 1)), hi = (int64_t(1) << (bits - 1)) - 1;
    return v >= lo && v <= hi;
}
inline int signed_bits_needed(int64_t v) {  // minimal two's complement width
    int b = 1;
    while (!fits(v, b)) b++;
    return b;
}

struct Encoder {
    const flacgen_config& c;
    int sbits;  // SampleType width 8/16/32
    int ibits;  // InterType width 16/32/64
    uint64_t partition_counter = 0;
    uint64_t subframe_counter = 0;
    int fault = 0;  // active fault kind for the frame being written
    bool force_verbatim = false;  // the subframe being written must be VERBATIM (planted sync)

    explicit Encoder(const flacgen_config& cfg) : c(cfg) {
        int aligned = (cfg.bps + 7) / 8 * 8;
        if (aligned == 8) { sbits = 8; ibits = 16; }
        else if (aligned == 16) { sbits = 16; ibits = 32; }
        else { sbits = 32; ibits = 64; }
    }

    // ---- residual coding -------------------------------------------------
    void write_residual(BitWriter& bw, const std::vector<int64_t>& r, int bs, int order) {
        int po = std::max(0, std::min(c.partition_order, 15));
        while (po > 0 && (((bs >> po) << po) != bs || (bs >> po) < order)) po--;
        const int np = 1 << po, psize = bs >> po;
        struct Part { int k; bool esc; int width; };
        std::vector<Part> parts(np);
        bool need_rice2 = c.rice2 != 0;
        size_t idx = 0;
        for (int p = 0; p < np; p++) {
            const int n = psize - (p == 0 ? order : 0);
            uint64_t sum = 0, maxzz = 0;
            int64_t maxabs = 0;
            for (int i = 0; i < n; i++) {
                const int64_t v = r[idx + i];
                const uint64_t zz = v >= 0 ? (uint64_t)v << 1 : (((uint64_t)(-(v + 1))) << 1) | 1;
                sum += zz;
                maxzz = std::max(maxzz, zz);
                maxabs = std::max(maxabs, v < 0 ? -(v + 1) : v);
            }
            Part pt{0, false, 0};
            const bool force_esc = c.escape_every > 0 && (partition_counter++ % c.escape_every) == 0;
            if (force_esc) {
                int w = 0;
                for (int i = 0; i < n; i++) w = std::max(w, r[idx + i] ? signed_bits_needed(r[idx + i]) : 0);
                if (w <= 31 && w <= ibits) { pt.esc = true; pt.width = w; }
            }
            if (!pt.esc) {
                int kmax = (ibits == 16) ? 15 : 30;
                if (c.rice_k >= 0) {
                    pt.k = std::min(c.rice_k, kmax);
                } else {
                    // best k by exact cost around the mean estimate
                    int k0 = 0;
                    if (n > 0) {
                        double mean = double(sum) / n;
                        while (k0 < kmax && double(1ull << (k0 + 1)) <= mean) k0++;
                    }
                    uint64_t best = ~0ull;
                    for (int k = std::max(0, k0 - 2); k <= std::min(kmax, k0 + 2); k++) {
                        uint64_t cost = uint64_t(n) * (k + 1);
                        for (int i = 0; i < n; i++) {
                            const int64_t v = r[idx + i];
                            const uint64_t zz = v >= 0 ? (uint64_t)v << 1 : (((uint64_t)(-(v + 1))) << 1) | 1;
                            cost += zz >> k;
                        }
                        if (cost < best) { best = cost; pt.k = k; }
                    }
                }
                // a quotient that large is technically fine but absurdly slow; keep codes sane
                while (pt.k < kmax && n > 0 && (maxzz >> pt.k) > 4096) pt.k++;
                if (pt.k > 14) need_rice2 = true;
            }
            (void)maxabs;
            parts[p] = pt;
            idx += n;
        }
        const int method = need_rice2 ? 1 : 0;
        bw.put(fault == 2 ? 2 : method, 2);
        if (fault == 5 && po == 0 && bs >= 2 * order + 2 && (bs & 1)) po = 1;  // 2^po does not divide bs
        bw.put(po, 4);
        if (fault == 5) fault = 0;
        idx = 0;
        for (int p = 0; p < np; p++) {
            const int n = psize - (p == 0 ? order : 0);
            const Part& pt = parts[p];
            if (pt.esc) {
                bw.put(method ? 31 : 15, method ? 5 : 4);
                bw.put(pt.width, 5);
                if (pt.width)
                    for (int i = 0; i < n; i++) bw.put_signed(r[idx + i], pt.width);
            } else {
                bw.put(pt.k, method ? 5 : 4);
                for (int i = 0; i < n; i++) {
                    const int64_t v = r[idx + i];
                    const uint64_t zz = v >= 0 ? (uint64_t)v << 1 : (((uint64_t)(-(v + 1))) << 1) | 1;
                    bw.unary(zz >> pt.k);
                    if (pt.k) bw.put(zz & ((1ull << pt.k) - 1), pt.k);
                }
            }
            idx += n;
        }
    }

    // ---- LPC analysis ------------------------------------------------------
    // Returns quantized coefficients q[0..order-1] (q[j] multiplies s[i-1-j]) and shift.
    bool lpc_coefs(const std::vector<int64_t>& x, int order, int precision, std::vector<int64_t>& q, int& shift) {
        const int n = (int)x.size();
        std::vector<double> w(n), R(order + 1, 0.0);
        for (int i = 0; i < n; i++) {
            double t = (2.0 * i - (n - 1)) / (n + 1);
            w[i] = x[i] * (1.0 - t * t);  // Welch window
        }
        for (int l = 0; l <= order; l++) {
            double s = 0;
            for (int i = l; i < n; i++) s += w[i] * w[i - l];
            R[l] = s;
        }
        if (R[0] <= 0) return false;
        R[0] *= 1.0 + 1e-9;
        std::vector<double> a(order + 1, 0.0), tmp(order + 1);
        double err = R[0];
        for (int i = 1; i <= order; i++) {
            double acc = R[i];
            for (int j = 1; j < i; j++) acc -= a[j] * R[i - j];
            double k = acc / err;
            tmp = a;
            a[i] = k;
            for (int j = 1; j < i; j++) a[j] = tmp[j] - k * tmp[i - j];
            err *= (1.0 - k * k);
            if (err <= 0) err = 1e-9;
        }
        double cmax = 0;
        for (int j = 1; j <= order; j++) cmax = std::max(cmax, std::fabs(a[j]));
        int e = 0;
        if (cmax > 0) std::frexp(cmax, &e);
        shift = precision - 1 - e;
        shift = std::max(0, std::min(shift, std::min(c.max_shift, 15)));
        q.assign(order, 0);
        double ef = 0;
        const int64_t qmax = (int64_t(1) << (precision - 1)) - 1, qmin = -(int64_t(1) << (precision - 1));
        for (int j = 0; j < order; j++) {
            double v = a[j + 1] * std::ldexp(1.0, shift) + ef;
            int64_t qi = std::llround(v);
            qi = std::max(qmin, std::min(qmax, qi));
            ef = v - double(qi);
            q[j] = qi;
        }
        return true;
    }

    // Residuals of s under reversed-coefficient prediction, verifying zflac's
    // InterType accumulation order (src/zflac.zig:527-532) never overflows.
    bool predict(const std::vector<int64_t>& s, int order, const std::vector<int64_t>& q, int shift,
                 std::vector<int64_t>& r) {
        const int n = (int)s.size();
        r.assign(n - order, 0);
        for (int i = order; i < n; i++) {
            int64_t p = 0;
            for (int o = 0; o < order; o++) {  // o indexes oldest-first, coef reversed
                const int64_t prod = s[i - order + o] * q[order - 1 - o];
                if (!fits(prod, ibits)) return false;
                p += prod;
                if (!fits(p, ibits)) return false;
            }
            const int64_t pred = p >> shift;
            const int64_t res = s[i] - pred;
            if (!fits(res, ibits)) return false;
            r[i - order] = res;
        }
        return true;
    }

    template <typename H>
    void write_fixed_or_verbatim(BitWriter& bw, const std::vector<int64_t>& u, int cbps, int bs, H& header) {
        std::vector<int64_t> q = {2, -1}, r;
        if (bs > 2 && predict(u, 2, q, 0, r)) {
            header(10);
            for (int i = 0; i < 2; i++) bw.put_signed(u[i], cbps);
            write_residual(bw, r, bs, 2);
            return;
        }
        header(1);
        for (int i = 0; i < bs; i++) bw.put_signed(u[i], cbps);
    }

    // ---- one subframe --------------------------------------------------------
    // v: the channel samples (after stereo transform), ubps: its coded width
    void write_subframe(BitWriter& bw, const std::vector<int64_t>& v, int ubps, bool side, int bs) {
        const uint64_t sf_index = subframe_counter++;
        // wasted bits: common trailing zeros
        uint64_t orv = 0;
        bool all_equal = true;
        for (int i = 0; i < bs; i++) {
            orv |= (uint64_t)v[i];
            all_equal &= v[i] == v[0];
        }
        int wasted = 0;
        if (orv) {
            while (!((orv >> wasted) & 1)) wasted++;
            wasted = std::min(wasted, ubps - 1);
            wasted = std::min(wasted, sbits - 1);
        }
        std::vector<int64_t> u(bs);
        for (int i = 0; i < bs; i++) u[i] = v[i] >> wasted;
        const int cbps = ubps - wasted;  // coded width of warm-up / verbatim samples

        auto header = [&](int type) {
            bw.put(0, 1);
            bw.put(fault == 1 ? 2 : type, 6);
            if (wasted) {
                bw.put(1, 1);
                bw.unary(wasted - 1);
            } else {
                bw.put(0, 1);
            }
        };
        // CONSTANT: zflac reads `bits_per_sample - wasted` bits, not the side width (:447);
        // an RFC encoder writes the side width (const_side == 2)
        const int const_bits = (ubps - (side && c.const_side != 2 ? 1 : 0)) - wasted;
        if (all_equal && !force_verbatim && (!side || c.const_side) && const_bits > 0 && fits(u[0], const_bits)) {
            header(0);
            bw.put_signed(u[0], const_bits);
            return;
        }
        const bool verbatim = force_verbatim || c.predictor == FG_VERBATIM ||
                              (c.verbatim_every > 0 && (sf_index % (uint64_t)c.verbatim_every) == 0);
        if (!verbatim) {
            int order = std::min(c.order, bs);
            if (c.predictor == FG_LPC && order >= 1 && (fault == 7 || fault == 8)) {
                // largest coefficients of the precision, shift 15: sum |c| * 2^(SB-1) exceeds
                // what the fast path proves safe; kind 8 keeps overflowing sums
                const int prec = c.precision;
                std::vector<int64_t> q(order, (int64_t(1) << (prec - 1)) - 1), r;
                const int shift = 15;
                if (!predict(u, order, q, shift, r)) {
                    if (fault == 7) return write_fixed_or_verbatim(bw, u, cbps, bs, header);
                    r.assign(bs - order, 0);
                    for (int i = order; i < bs; i++) {
                        __int128 p = 0;
                        for (int o = 0; o < order; o++) p += (__int128)u[i - order + o] * q[order - 1 - o];
                        const __int128 res = (__int128)u[i] - (p >> shift);
                        r[i - order] = fits((int64_t)res, ibits) && res == (__int128)(int64_t)res ? (int64_t)res : 0;
                    }
                }
                header(31 + order);
                for (int i = 0; i < order; i++) bw.put_signed(u[i], cbps);
                bw.put(prec - 1, 4);
                bw.put(shift, 5);
                for (int j = 0; j < order; j++) bw.put_signed(q[j], prec);
                write_residual(bw, r, bs, order);
                return;
            }
            if (c.predictor == FG_LPC && order >= 1) {
                for (int prec = c.precision; prec >= 1; prec--) {
                    std::vector<int64_t> q, r;
                    int shift = 0;
                    if (!lpc_coefs(u, order, prec, q, shift)) break;
                    if (!predict(u, order, q, shift, r)) continue;
                    header(31 + order);
                    for (int i = 0; i < order; i++) bw.put_signed(u[i], cbps);
                    bw.put(fault == 3 ? 15 : prec - 1, 4);
                    bw.put(shift, 5);
                    for (int j = 0; j < order; j++) bw.put_signed(q[j], prec);
                    write_residual(bw, r, bs, order);
                    return;
                }
                // fall through to fixed order 2
                order = std::min(2, bs);
            }
            order = std::min(order, 4);
            static const int64_t F[5][4] = {{0}, {1}, {2, -1}, {3, -3, 1}, {4, -6, 4, -1}};
            std::vector<int64_t> q(F[order], F[order] + order), r;
            if (predict(u, order, q, 0, r)) {
                header(8 + order);
                for (int i = 0; i < order; i++) bw.put_signed(u[i], cbps);
                write_residual(bw, r, bs, order);
                return;
            }
        }
        header(1);
        for (int i = 0; i < bs; i++) bw.put_signed(u[i], cbps);
    }
};

void put_utf8_number(std::vector<uint8_t>& h, uint64_t v) {
    if (v < 0x80) { h.push_back((uint8_t)v); return; }
    int nbytes = 2;
    while (nbytes < 7 && v >= (1ull << (5 * nbytes + 1))) nbytes++;
    const uint8_t lead_mask = (uint8_t)(0xFF00 >> nbytes);
    h.push_back((uint8_t)(lead_mask | (v >> (6 * (nbytes - 1)))));
    for (int i = nbytes - 2; i >= 0; i--) h.push_back((uint8_t)(0x80 | ((v >> (6 * i)) & 0x3F)));
}

int block_size_code(int bs, int& extra_bits) {
    extra_bits = 0;
    if (bs == 192) return 1;
    for (int b = 2; b <= 5; b++) if (bs == (144 << b)) return b;
    for (int b = 8; b <= 15; b++) if (bs == (1 << b)) return b;
    if (bs <= 256) { extra_bits = 8; return 6; }
    extra_bits = 16;
    return 7;
}

int rate_code(int rate, int mode, int& extra_bits, int& extra_val) {
    extra_bits = 0;
    extra_val = 0;
    if (mode == 3) return 0;
    static const int T[12] = {0, 88200, 176400, 192000, 8000, 16000, 22050, 24000, 32000, 44100, 48000, 96000};
    if (mode == 0)
        for (int i = 1; i < 12; i++) if (T[i] == rate) return i;
    if (mode == 2 && rate % 10 == 0 && rate / 10 <= 0xFFFF) { extra_bits = 16; extra_val = rate / 10; return 14; }
    if (rate <= 0xFFFF) { extra_bits = 16; extra_val = rate; return 13; }
    return 0;  // stored in STREAMINFO
}

int depth_code(int bps) {
    switch (bps) {
        case 8: return 1;
        case 12: return 2;
        case 16: return 4;
        case 20: return 5;
        case 24: return 6;
        case 32: return 7;
        default: return 0;
    }
}

// Frame header with CRC-8 (RFC 9639 11.21; parsed by zflac at src/zflac.zig:343-407)
std::vector<uint8_t> frame_header(const flacgen_config& c, size_t f, int bs, int chan_code, uint64_t sample_no) {
    int bx, rx, rv;
    std::vector<uint8_t> h;
    h.push_back(0xFF);
    h.push_back(c.variable_blocking ? 0xF9 : 0xF8);
    const int bsc = block_size_code(bs, bx);
    const int rc = rate_code(c.sample_rate, c.rate_code_mode, rx, rv);
    h.push_back((uint8_t)((bsc << 4) | rc));
    h.push_back((uint8_t)((chan_code << 4) | (depth_code(c.bps) << 1)));
    put_utf8_number(h, c.variable_blocking ? sample_no : (uint64_t)f);
    if (bx == 8) h.push_back((uint8_t)(bs - 1));
    if (bx == 16) { h.push_back((uint8_t)((bs - 1) >> 8)); h.push_back((uint8_t)(bs - 1)); }
    if (rx == 16) { h.push_back((uint8_t)(rv >> 8)); h.push_back((uint8_t)rv); }
    h.push_back(crc8(h.data(), h.size()));
    return h;
}

struct Synth {
    // sum of sinusoids (recursive oscillators) + first-order coloured noise
    struct Osc { double c, s, cr, sr, amp; };
    std::vector<Osc> osc;
    double ar = 0;
    Rng rng;
    Synth(uint64_t seed, int ntones, double total_amp) : rng(seed) {
        for (int i = 0; i < ntones; i++) {
            double f = 0.002 + 0.08 * rng.uniform();  // cycles/sample
            double ph = 6.283185307179586 * rng.uniform();
            double w = 6.283185307179586 * f;
            osc.push_back({std::cos(ph), std::sin(ph), std::cos(w), std::sin(w), total_amp / ntones * (0.5 + rng.uniform())});
        }
    }
    double tone() {
        double v = 0;
        for (auto& o : osc) {
            v += o.amp * o.s;
            double nc = o.c * o.cr - o.s * o.sr, ns = o.s * o.cr + o.c * o.sr;
            o.c = nc;
            o.s = ns;
        }
        return v;
    }
    double noise() {
        ar = 0.6 * ar + rng.gauss();
        return ar * 0.8;
    }
};

}  // namespace

extern "C" {

void flacgen_default_config(flacgen_config* c) {
    std::memset(c, 0, sizeof(*c));
    c->channels = 2;
    c->bps = 16;
    c->block_size = 4096;
    c->predictor = FG_LPC;
    c->order = 8;
    c->precision = 12;
    c->max_shift = 15;
    c->stereo_mode = 10;
    c->partition_order = 4;
    c->rice_k = -1;
    c->sample_rate = 44100;
    c->write_total = 1;
    c->tone_amp = 0.25;
    c->noise_lsb = 64.0;
    c->stereo_corr = 0.8;
    c->n_samples = 4096 * 8;
    c->seed = 1;
    c->fault_frame = -1;
}

static int generate_impl(const flacgen_config* cfg, const int32_t* ext_pcm, flacgen_output* out) {
    std::memset(out, 0, sizeof(*out));
    const flacgen_config& c = *cfg;
    if (c.channels < 1 || c.channels > 8 || c.bps < 4 || c.bps > 32 || c.block_size < 16 || c.block_size > 65535)
        return -1;
    if (c.predictor == FG_LPC && (c.order < 1 || c.order > 32 || c.precision < 1 || c.precision > 15)) return -1;
    if (c.predictor == FG_FIXED && (c.order < 0 || c.order > 4)) return -1;
    if (c.plant_sync_every > 0 && ((c.bps != 8 && c.bps != 16 && c.bps != 24) || c.wasted_bits ||
                                   (c.channels == 2 && c.stereo_mode != 1)))
        return -1;  // the planted header must sit byte-aligned in a VERBATIM channel-0 subframe
    Encoder enc(c);
    const int C = c.channels;
    const int sig_bits = c.bps - c.wasted_bits;  // significant bits
    if (sig_bits < 2) return -1;
    const double fs = std::ldexp(1.0, sig_bits - 1);
    const int64_t smax = (int64_t(1) << (sig_bits - 1)) - 1, smin = -(int64_t(1) << (sig_bits - 1));

    std::vector<Synth> syn;
    for (int ch = 0; ch < C; ch++) syn.emplace_back(c.seed * 131 + ch * 7 + 11, 4 + (int)(c.seed % 5), c.tone_amp);
    Rng brng(c.seed ^ 0xB10C);

    // block sizes
    std::vector<int> blocks;
    uint64_t left = c.n_samples;
    while (left > 0) {
        int bs = c.block_size;
        if (c.variable_blocking) bs = 16 + (int)(brng.next() % (uint64_t)std::max(1, c.block_size - 15));
        if ((uint64_t)bs > left) bs = (int)left;
        blocks.push_back(bs);
        left -= bs;
    }
    if (c.fault_kind == 4 && c.fault_frame >= 0 && (size_t)c.fault_frame < blocks.size() &&
        (size_t)c.fault_frame + 1 < blocks.size()) {
        blocks[c.fault_frame] -= 1;
        blocks.insert(blocks.begin() + c.fault_frame + 1, 1);
    }
    std::vector<uint8_t> frames;
    std::vector<uint64_t> frame_offs;
    std::vector<int32_t> pcm;
    pcm.reserve(c.n_samples * C);
    zflac::Md5 md5;
    const int md5_bytes = (c.bps + 7) / 8;
    uint32_t min_frame = ~0u, max_frame = 0;
    int min_block = 65535, max_block = 0;
    uint64_t sample_no = 0;

    for (size_t f = 0; f < blocks.size(); f++) {
        const int bs = blocks[f];
        // --- synthesize -----------------------------------------------------
        std::vector<std::vector<int64_t>> x(C, std::vector<int64_t>(bs));
        const bool silent0 = c.silence_every > 0 && (f % (size_t)c.silence_every) == 0;
        const bool dual = C >= 2 && c.dual_mono_every > 0 && (f % (size_t)c.dual_mono_every) == (size_t)c.dual_mono_every - 1;
        for (int i = 0; i < bs; i++) {
            if (ext_pcm) {
                for (int ch = 0; ch < C; ch++) x[ch][i] = ext_pcm[(sample_no + i) * C + ch];
                continue;
            }
            double base = syn[0].tone() * fs + syn[0].noise() * c.noise_lsb;
            for (int ch = 0; ch < C; ch++) {
                double v;
                if (ch == 0) v = base;
                else v = c.stereo_corr * base + (1.0 - c.stereo_corr) * syn[ch].tone() * fs + syn[ch].noise() * c.noise_lsb;
                int64_t q = std::llround(v);
                q = std::max(smin, std::min(smax, q));
                if (ch == 0 && silent0) q = 0;
                if (ch == 1 && dual) q = std::max(smin, std::min(smax, x[0][i] / (int64_t(1) << c.wasted_bits) - c.dual_mono_offset));
                x[ch][i] = q * (int64_t(1) << c.wasted_bits);
            }
        }
        // planted false sync: channel 0 (VERBATIM, byte-aligned samples) carries a copy of
        // this frame's own header, CRC-8 included, from sample bs / 2 on
        const bool plant = c.plant_sync_every > 0 && (f % (size_t)c.plant_sync_every) == (size_t)c.plant_sync_every - 1;
        if (plant) {
            const std::vector<uint8_t> h = frame_header(c, f, bs, C == 1 ? 0 : C - 1, sample_no);
            const int B = c.bps / 8;
            const int i0 = bs / 2;
            const int n = ((int)h.size() + B - 1) / B;
            if (i0 < 1 || i0 + n > bs) return -1;
            for (int j = 0; j < n; j++) {
                uint64_t v = 0;
                for (int b = 0; b < B; b++) {
                    const size_t k = (size_t)j * B + b;
                    v = (v << 8) | (k < h.size() ? h[k] : 0x55);
                }
                x[0][i0 + j] = (int64_t)(v << (64 - 8 * B)) >> (64 - 8 * B);
            }
            x[0][i0 - 1] |= 1;  // no wasted bits: the samples stay byte-aligned
        }
        for (int i = 0; i < bs; i++)
            for (int ch = 0; ch < C; ch++) {
                pcm.push_back((int32_t)x[ch][i]);
                uint8_t b[4];
                uint32_t u = (uint32_t)(int32_t)x[ch][i];
                for (int k = 0; k < 4; k++) b[k] = (uint8_t)(u >> (8 * k));
                md5.update(b, md5_bytes);
            }
        // --- stereo decorrelation choice -------------------------------------
        int chan_code = C - 1;
        std::vector<std::vector<int64_t>> sub = x;
        std::vector<int> ubps(C, c.bps);
        std::vector<bool> side(C, false);
        if (C == 2) {
            auto make = [&](int mode, std::vector<std::vector<int64_t>>& s, bool& ok) {
                s.assign(2, std::vector<int64_t>(bs));
                ok = true;
                for (int i = 0; i < bs; i++) {
                    int64_t L = x[0][i], R = x[1][i], S = L - R;
                    if (mode != 1 && !fits(S, enc.sbits) && !c.allow_side_overflow) ok = false;
                    if (mode == 1) { s[0][i] = L; s[1][i] = R; }
                    else if (mode == 8) { s[0][i] = L; s[1][i] = S; }
                    else if (mode == 9) { s[0][i] = S; s[1][i] = R; }
                    else { s[0][i] = (L + R) >> 1; s[1][i] = S; }
                }
            };
            int mode = c.stereo_mode;
            if (mode == -1) {
                double best = 1e300;
                for (int m : {1, 8, 9, 10}) {
                    std::vector<std::vector<int64_t>> s;
                    bool ok;
                    make(m, s, ok);
                    if (!ok) continue;
                    double cost = 0;
                    for (int ch = 0; ch < 2; ch++)
                        for (int i = 2; i < bs; i++) cost += std::fabs(double(s[ch][i] - 2 * s[ch][i - 1] + s[ch][i - 2]));
                    if (cost < best) { best = cost; mode = m; }
                }
            }
            bool ok;
            make(mode, sub, ok);
            if (!ok) return -2;  // side channel does not fit the SampleType container
            chan_code = mode == 1 ? 1 : mode;
            if (mode == 8 || mode == 10) { ubps[1] = c.bps + 1; side[1] = true; }
            if (mode == 9) { ubps[0] = c.bps + 1; side[0] = true; }
        }
        if (c.fault_kind == 6 && (int)f == c.fault_frame)  // decorrelation overflow (stereo)
            for (int i = 0; i < bs; i++) sub[0][i] = (int64_t(1) << (enc.sbits - 1)) - 1;
        // --- header -----------------------------------------------------------
        BitWriter bw;
        bw.buf = frame_header(c, f, bs, chan_code, sample_no);
        for (int ch = 0; ch < C; ch++) {
            enc.fault = (ch == 0 && (int)f == c.fault_frame && c.fault_kind != 4 && c.fault_kind != 6) ? c.fault_kind : 0;
            enc.force_verbatim = plant && ch == 0;
            enc.write_subframe(bw, sub[ch], ubps[ch], side[ch], bs);
            enc.fault = 0;
            enc.force_verbatim = false;
        }
        bw.align();
        uint16_t crc = crc16(bw.buf.data(), bw.buf.size());
        bw.put(crc, 16);
        frame_offs.push_back(frames.size());
        min_frame = std::min<uint32_t>(min_frame, (uint32_t)bw.buf.size());
        max_frame = std::max<uint32_t>(max_frame, (uint32_t)bw.buf.size());
        if (f + 1 < blocks.size() || blocks.size() == 1) min_block = std::min(min_block, bs);
        max_block = std::max(max_block, bs);
        frames.insert(frames.end(), bw.buf.begin(), bw.buf.end());
        sample_no += bs;
    }
    md5.finish(out->md5);

    // --- stream: signature + metadata ------------------------------------------
    std::vector<uint8_t> s = {'f', 'L', 'a', 'C'};
    std::vector<std::vector<uint8_t>> blocks_md;
    std::vector<int> types;
    {
        BitWriter si;
        si.put(c.variable_blocking ? (uint64_t)std::min(min_block, 65535) : (uint64_t)c.block_size, 16);
        si.put(c.variable_blocking ? (uint64_t)max_block : (uint64_t)c.block_size, 16);
        si.put(min_frame == ~0u ? 0 : min_frame, 24);
        si.put(max_frame, 24);
        si.put((uint64_t)c.sample_rate, 20);
        si.put(C - 1, 3);
        si.put(c.bps - 1, 5);
        si.put(c.write_total ? c.n_samples : 0, 36);
        for (int i = 0; i < 16; i++) si.put(out->md5[i], 8);
        blocks_md.push_back(si.buf);
        types.push_back(0);
    }
    if (c.extra_metadata) {
        std::vector<uint8_t> app = {'z', 'f', 'h', 'p', 1, 2, 3, 4, 5};
        blocks_md.push_back(app);
        types.push_back(2);
        std::vector<uint8_t> seek;
        for (int p = 0; p < 2; p++) {
            uint64_t sn = p == 0 ? 0 : 0xFFFFFFFFFFFFFFFFull;  // second is a placeholder point
            for (int i = 7; i >= 0; i--) seek.push_back((uint8_t)(sn >> (8 * i)));
            for (int i = 7; i >= 0; i--) seek.push_back(0);
            seek.push_back(0x10);
            seek.push_back(0x00);
        }
        blocks_md.push_back(seek);
        types.push_back(3);
        const char* vendor = "flacgen synthetic";
        std::vector<uint8_t> vc;
        uint32_t vl = (uint32_t)std::strlen(vendor);
        for (int i = 0; i < 4; i++) vc.push_back((uint8_t)(vl >> (8 * i)));
        vc.insert(vc.end(), vendor, vendor + vl);
        for (int i = 0; i < 4; i++) vc.push_back(0);
        blocks_md.push_back(vc);
        types.push_back(4);
        blocks_md.push_back(std::vector<uint8_t>(37, 0));
        types.push_back(1);
    }
    for (size_t b = 0; b < blocks_md.size(); b++) {
        const uint32_t len = (uint32_t)blocks_md[b].size();
        s.push_back((uint8_t)(((b + 1 == blocks_md.size()) ? 0x80 : 0) | types[b]));
        s.push_back((uint8_t)(len >> 16));
        s.push_back((uint8_t)(len >> 8));
        s.push_back((uint8_t)len);
        s.insert(s.end(), blocks_md[b].begin(), blocks_md[b].end());
    }
    out->frames_begin = s.size();
    s.insert(s.end(), frames.begin(), frames.end());

    out->flac_len = s.size();
    out->flac = (uint8_t*)std::malloc(s.size());
    std::memcpy(out->flac, s.data(), s.size());
    out->pcm_len = pcm.size();
    out->pcm = (int32_t*)std::malloc(std::max<size_t>(1, pcm.size() * sizeof(int32_t)));
    if (!pcm.empty()) std::memcpy(out->pcm, pcm.data(), pcm.size() * sizeof(int32_t));
    out->n_frames = (uint32_t)frame_offs.size();
    out->frame_offsets = (uint64_t*)std::malloc(std::max<size_t>(1, frame_offs.size() * sizeof(uint64_t)));
    for (size_t i = 0; i < frame_offs.size(); i++) out->frame_offsets[i] = frame_offs[i] + out->frames_begin;
    return 0;
}

int flacgen_generate(const flacgen_config* cfg, flacgen_output* out) { return generate_impl(cfg, nullptr, out); }

int flacgen_generate_pcm(const flacgen_config* cfg, const int32_t* pcm, uint64_t len, flacgen_output* out) {
    if (!pcm || cfg->channels < 1 || len % (uint64_t)cfg->channels) return -1;
    flacgen_config c = *cfg;
    c.n_samples = len / (uint64_t)cfg->channels;
    const int64_t lo = -(int64_t(1) << (c.bps - 1)), hi = (int64_t(1) << (c.bps - 1)) - 1;
    for (uint64_t i = 0; i < len; i++)
        if (pcm[i] < lo || pcm[i] > hi) return -1;
    return generate_impl(&c, pcm, out);
}

void flacgen_free(flacgen_output* out) {
    if (!out) return;
    std::free(out->flac);
    std::free(out->pcm);
    std::free(out->frame_offsets);
    out->flac = nullptr;
    out->pcm = nullptr;
    out->frame_offsets = nullptr;
}

}  // extern "C"
