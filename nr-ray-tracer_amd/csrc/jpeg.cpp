// Baseline / extended-sequential Huffman JPEG decoder for image textures
// (Image::try_from_path -> into_rgb32f, lib/textures/image.rs:24-28).
//
// The reference decodes with the `image` crate 0.25.8, which uses zune-jpeg
// 0.4.21 (Cargo.lock); neither is available here.  This decoder follows
// libjpeg's defaults instead -- the accurate integer IDCT (jidctint.c
// "islow": 13-bit constants, 2 pass-1 bits, the post-IDCT range-limit table)
// and the table-driven YCbCr -> RGB conversion of jdcolor.c (16-bit fixed
// point) -- so its samples equal libjpeg-turbo's (PIL, used by the oracle's
// loader) bit for bit on 4:4:4 files such as the reference's earth.jpg and
// moon.jpg.  Against zune-jpeg the parity is unpinned (its IDCT and colour
// conversion are separate integer approximations).  Chroma-subsampled files are
// upsampled by replication (libjpeg's default "fancy" triangle filter is not
// reproduced); progressive and arithmetic-coded files are rejected.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "scene_config.hpp"

namespace nrt {

namespace {

// Natural order of the zig-zag coefficient sequence.
const uint8_t ZIGZAG[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                            12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                            35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                            58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huffman {
    bool present = false;
    // canonical code tables: codes of length L are [mincode[L], maxcode[L]], values from valptr[L]
    int32_t mincode[17], maxcode[18], valptr[17];
    uint8_t vals[256];
};

struct Component {
    int id = 0, h = 1, v = 1, tq = 0;
    int td = 0, ta = 0;  // Huffman table selectors (from SOS)
    int bw = 0, bh = 0;  // blocks per line / column (padded to whole MCUs)
    int pred = 0;        // DC predictor
    std::vector<uint8_t> samples;  // bw*8 x bh*8
};

struct Decoder {
    const uint8_t* d;
    size_t n, pos = 0;
    std::string err;
    uint16_t qt[4][64] = {};
    bool qt_present[4] = {};
    Huffman dc[4], ac[4];
    std::vector<Component> comps;
    int width = 0, height = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
    int restart_interval = 0;
    int adobe_transform = -1;  // APP14 "Adobe" transform flag, -1 = absent
    bool jfif = false;
    // entropy-coded segment bit reader
    uint32_t bitbuf = 0;
    int bitcnt = 0;
    bool hit_marker = false;

    bool fail(const std::string& m) {
        if (err.empty()) err = m;
        return false;
    }
    int u8() { return pos < n ? d[pos++] : (hit_marker = true, 0); }
    int u16() {
        const int a = u8();
        return (a << 8) | u8();
    }

    bool read_dqt(size_t end) {
        while (pos < end) {
            const int pq = d[pos] >> 4, tq = d[pos] & 15;
            ++pos;
            if (tq > 3) return fail("bad quantization table id");
            for (int k = 0; k < 64; ++k) qt[tq][ZIGZAG[k]] = (uint16_t)(pq ? u16() : u8());
            qt_present[tq] = true;
        }
        return true;
    }

    bool read_dht(size_t end) {
        while (pos < end) {
            const int tc = d[pos] >> 4, th = d[pos] & 15;
            ++pos;
            if (tc > 1 || th > 3 || pos + 16 > end) return fail("bad Huffman table");
            Huffman& h = tc == 0 ? dc[th] : ac[th];
            int counts[17] = {};
            int total = 0;
            for (int l = 1; l <= 16; ++l) total += counts[l] = d[pos++];
            if (total > 256 || pos + (size_t)total > end) return fail("bad Huffman table");
            for (int k = 0; k < total; ++k) h.vals[k] = d[pos++];
            int code = 0, k = 0;
            for (int l = 1; l <= 16; ++l) {
                h.valptr[l] = k;
                h.mincode[l] = code;
                code += counts[l];
                k += counts[l];
                h.maxcode[l] = counts[l] ? code - 1 : -1;
                code <<= 1;
            }
            h.maxcode[17] = 0x7FFFFFFF;
            h.present = true;
        }
        return true;
    }

    bool read_sof(size_t end) {
        if (u8() != 8) return fail("only 8-bit samples are supported");
        height = u16();
        width = u16();
        const int nc = u8();
        if (width <= 0 || height <= 0) return fail("bad image size");
        if (nc != 1 && nc != 3) return fail("only 1- or 3-component images are supported");
        comps.resize(nc);
        for (auto& c : comps) {
            c.id = u8();
            const int hv = u8();
            c.h = hv >> 4;
            c.v = hv & 15;
            c.tq = u8();
            if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3) return fail("bad component");
            hmax = std::max(hmax, c.h);
            vmax = std::max(vmax, c.v);
        }
        if (pos != end) return fail("bad SOF length");
        mcux = (width + 8 * hmax - 1) / (8 * hmax);
        mcuy = (height + 8 * vmax - 1) / (8 * vmax);
        for (auto& c : comps) {
            c.bw = mcux * c.h;
            c.bh = mcuy * c.v;
            c.samples.assign((size_t)c.bw * 8 * c.bh * 8, 0);
        }
        return true;
    }

    // ---- entropy decoding
    void fill() {
        while (bitcnt <= 24) {
            int byte = 0;
            if (!hit_marker && pos < n) {
                byte = d[pos];
                if (byte == 0xFF) {
                    const int next = pos + 1 < n ? d[pos + 1] : 0;
                    if (next == 0x00) {
                        pos += 2;
                    } else {  // a marker: feed zeros from here on
                        hit_marker = true;
                        byte = 0;
                    }
                } else {
                    ++pos;
                }
            }
            bitbuf |= (uint32_t)byte << (24 - bitcnt);
            bitcnt += 8;
        }
    }
    int bits(int k) {
        if (k == 0) return 0;
        fill();
        const int v = (int)(bitbuf >> (32 - k));
        bitbuf <<= k;
        bitcnt -= k;
        return v;
    }
    int decode(const Huffman& h) {
        fill();
        int code = 0;
        for (int l = 1; l <= 16; ++l) {
            code = (code << 1) | (int)(bitbuf >> 31);
            bitbuf <<= 1;
            --bitcnt;
            if (code <= h.maxcode[l]) return h.vals[h.valptr[l] + code - h.mincode[l]];
        }
        err = "corrupt Huffman code";
        return 0;
    }
    static int extend(int v, int t) { return v < (1 << (t - 1)) ? v - (1 << t) + 1 : v; }

    bool decode_block(Component& c, int16_t blk[64]) {
        std::memset(blk, 0, 64 * sizeof(int16_t));
        const int t = decode(dc[c.td]);
        if (t > 11) return fail("bad DC magnitude");
        const int diff = t ? extend(bits(t), t) : 0;
        c.pred += diff;
        blk[0] = (int16_t)c.pred;
        for (int k = 1; k < 64;) {
            const int rs = decode(ac[c.ta]);
            const int r = rs >> 4, sz = rs & 15;
            if (sz == 0) {
                if (r != 15) break;  // EOB
                k += 16;
                continue;
            }
            k += r;
            if (k > 63) return fail("bad AC run");
            blk[ZIGZAG[k]] = (int16_t)extend(bits(sz), sz);
            ++k;
        }
        return err.empty();
    }

    // ---- jidctint.c jpeg_idct_islow, output through the post-IDCT range-limit table
    static uint8_t range_limit_idct(int x) {  // x = DESCALE(...) (centred sample), table semantics & 1023
        const int i = x & 1023;
        if (i < 128) return (uint8_t)(i + 128);
        if (i < 512) return 255;
        if (i < 896) return 0;
        return (uint8_t)(i - 896);
    }
    static void idct_islow(const int16_t* in, const uint16_t* q, uint8_t* out, int stride) {
        typedef int64_t L;
        const int CB = 13, P1 = 2;
        auto descale = [](L x, int nbits) { return (L)((x + ((L)1 << (nbits - 1))) >> nbits); };
        const L F0_298 = 2446, F0_390 = 3196, F0_541 = 4433, F0_765 = 6270, F0_899 = 7373, F1_175 = 9633,
                F1_501 = 12299, F1_847 = 15137, F1_961 = 16069, F2_053 = 16819, F2_562 = 20995, F3_072 = 25172;
        int ws[64];
        for (int c = 0; c < 8; ++c) {  // pass 1: columns
            auto DQ = [&](int r) { return (L)in[8 * r + c] * (L)q[8 * r + c]; };
            if (in[8 + c] == 0 && in[16 + c] == 0 && in[24 + c] == 0 && in[32 + c] == 0 && in[40 + c] == 0 &&
                in[48 + c] == 0 && in[56 + c] == 0) {
                const int dcval = (int)(DQ(0) * (1 << P1));
                for (int r = 0; r < 8; ++r) ws[8 * r + c] = dcval;
                continue;
            }
            L z2 = DQ(2), z3 = DQ(6);
            L z1 = (z2 + z3) * F0_541;
            L tmp2 = z1 + z3 * -F1_847;
            L tmp3 = z1 + z2 * F0_765;
            z2 = DQ(0);
            z3 = DQ(4);
            L tmp0 = (z2 + z3) * (1 << CB);
            L tmp1 = (z2 - z3) * (1 << CB);
            const L tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
            tmp0 = DQ(7);
            tmp1 = DQ(5);
            tmp2 = DQ(3);
            tmp3 = DQ(1);
            z1 = tmp0 + tmp3;
            z2 = tmp1 + tmp2;
            z3 = tmp0 + tmp2;
            L z4 = tmp1 + tmp3;
            const L z5 = (z3 + z4) * F1_175;
            tmp0 *= F0_298;
            tmp1 *= F2_053;
            tmp2 *= F3_072;
            tmp3 *= F1_501;
            z1 *= -F0_899;
            z2 *= -F2_562;
            z3 *= -F1_961;
            z4 *= -F0_390;
            z3 += z5;
            z4 += z5;
            tmp0 += z1 + z3;
            tmp1 += z2 + z4;
            tmp2 += z2 + z3;
            tmp3 += z1 + z4;
            ws[c] = (int)descale(tmp10 + tmp3, CB - P1);
            ws[56 + c] = (int)descale(tmp10 - tmp3, CB - P1);
            ws[8 + c] = (int)descale(tmp11 + tmp2, CB - P1);
            ws[48 + c] = (int)descale(tmp11 - tmp2, CB - P1);
            ws[16 + c] = (int)descale(tmp12 + tmp1, CB - P1);
            ws[40 + c] = (int)descale(tmp12 - tmp1, CB - P1);
            ws[24 + c] = (int)descale(tmp13 + tmp0, CB - P1);
            ws[32 + c] = (int)descale(tmp13 - tmp0, CB - P1);
        }
        for (int r = 0; r < 8; ++r) {  // pass 2: rows
            const int* w = ws + 8 * r;
            uint8_t* o = out + (size_t)r * stride;
            if (w[1] == 0 && w[2] == 0 && w[3] == 0 && w[4] == 0 && w[5] == 0 && w[6] == 0 && w[7] == 0) {
                const uint8_t dcval = range_limit_idct((int)descale(w[0], P1 + 3));
                for (int c = 0; c < 8; ++c) o[c] = dcval;
                continue;
            }
            L z2 = w[2], z3 = w[6];
            L z1 = (z2 + z3) * F0_541;
            L tmp2 = z1 + z3 * -F1_847;
            L tmp3 = z1 + z2 * F0_765;
            L tmp0 = ((L)w[0] + (L)w[4]) * (1 << CB);
            L tmp1 = ((L)w[0] - (L)w[4]) * (1 << CB);
            const L tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
            tmp0 = w[7];
            tmp1 = w[5];
            tmp2 = w[3];
            tmp3 = w[1];
            z1 = tmp0 + tmp3;
            z2 = tmp1 + tmp2;
            z3 = tmp0 + tmp2;
            L z4 = tmp1 + tmp3;
            const L z5 = (z3 + z4) * F1_175;
            tmp0 *= F0_298;
            tmp1 *= F2_053;
            tmp2 *= F3_072;
            tmp3 *= F1_501;
            z1 *= -F0_899;
            z2 *= -F2_562;
            z3 *= -F1_961;
            z4 *= -F0_390;
            z3 += z5;
            z4 += z5;
            tmp0 += z1 + z3;
            tmp1 += z2 + z4;
            tmp2 += z2 + z3;
            tmp3 += z1 + z4;
            const int S = CB + P1 + 3;
            o[0] = range_limit_idct((int)descale(tmp10 + tmp3, S));
            o[7] = range_limit_idct((int)descale(tmp10 - tmp3, S));
            o[1] = range_limit_idct((int)descale(tmp11 + tmp2, S));
            o[6] = range_limit_idct((int)descale(tmp11 - tmp2, S));
            o[2] = range_limit_idct((int)descale(tmp12 + tmp1, S));
            o[5] = range_limit_idct((int)descale(tmp12 - tmp1, S));
            o[3] = range_limit_idct((int)descale(tmp13 + tmp0, S));
            o[4] = range_limit_idct((int)descale(tmp13 - tmp0, S));
        }
    }

    bool read_restart() {  // byte-align, expect RSTn
        bitbuf = 0;
        bitcnt = 0;
        hit_marker = false;
        while (pos + 1 < n && !(d[pos] == 0xFF && d[pos + 1] >= 0xD0 && d[pos + 1] <= 0xD7)) ++pos;
        if (pos + 1 >= n) return fail("missing restart marker");
        pos += 2;
        for (auto& c : comps) c.pred = 0;
        return true;
    }

    bool read_sos(size_t end) {
        const int ns = u8();
        if (ns < 1 || ns > (int)comps.size()) return fail("bad scan");
        std::vector<Component*> sc;
        for (int k = 0; k < ns; ++k) {
            const int id = u8(), t = u8();
            Component* c = nullptr;
            for (auto& x : comps)
                if (x.id == id) c = &x;
            if (!c) return fail("scan names an unknown component");
            c->td = t >> 4;
            c->ta = t & 15;
            if (c->td > 3 || c->ta > 3 || !dc[c->td].present || !ac[c->ta].present || !qt_present[c->tq])
                return fail("scan uses a missing table");
            sc.push_back(c);
        }
        const int ss = u8(), se = u8(), ahal = u8();
        if (ss != 0 || se != 63 || ahal != 0) return fail("progressive scans are not supported");
        pos = end;
        bitbuf = 0;
        bitcnt = 0;
        hit_marker = false;
        for (auto* c : sc) c->pred = 0;
        int16_t blk[64];
        auto put = [&](Component& c, int bx, int by) {
            if (!decode_block(c, blk)) return false;
            const int stride = c.bw * 8;
            idct_islow(blk, qt[c.tq], c.samples.data() + (size_t)by * 8 * stride + (size_t)bx * 8, stride);
            return true;
        };
        int todo = restart_interval;
        if (ns == 1) {  // non-interleaved: the component's own block grid (no padding blocks)
            Component& c = *sc[0];
            const int cw = (width * c.h + 8 * hmax - 1) / (8 * hmax), ch = (height * c.v + 8 * vmax - 1) / (8 * vmax);
            for (int by = 0; by < ch; ++by)
                for (int bx = 0; bx < cw; ++bx) {
                    if (restart_interval && todo == 0) {
                        if (!read_restart()) return false;
                        todo = restart_interval;
                    }
                    if (!put(c, bx, by)) return false;
                    --todo;
                }
        } else {
            for (int my = 0; my < mcuy; ++my)
                for (int mx = 0; mx < mcux; ++mx) {
                    if (restart_interval && todo == 0) {
                        if (!read_restart()) return false;
                        todo = restart_interval;
                    }
                    for (auto* c : sc)
                        for (int v = 0; v < c->v; ++v)
                            for (int h = 0; h < c->h; ++h)
                                if (!put(*c, mx * c->h + h, my * c->v + v)) return false;
                    --todo;
                }
        }
        // resume marker parsing at the next marker
        while (pos + 1 < n && !(d[pos] == 0xFF && d[pos + 1] != 0x00 && !(d[pos + 1] >= 0xD0 && d[pos + 1] <= 0xD7)))
            ++pos;
        return true;
    }

    bool run(DecodedImage& out) {
        if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return fail("not a JPEG file");
        pos = 2;
        bool frame = false, scanned = false;
        while (pos + 4 <= n) {
            if (d[pos] != 0xFF) return fail("marker expected");
            while (pos < n && d[pos] == 0xFF) ++pos;  // fill bytes
            if (pos >= n) return fail("truncated marker");
            const int m = d[pos++];
            if (m == 0xD9) break;  // EOI
            if (m >= 0xD0 && m <= 0xD7) continue;
            const size_t len = (size_t)u16();
            if (len < 2 || pos - 2 + len > n) return fail("truncated segment");
            const size_t end = pos - 2 + len;
            bool ok = true;
            switch (m) {
                case 0xC0:
                case 0xC1:  // baseline / extended sequential, Huffman
                    ok = !frame && read_sof(end);
                    frame = true;
                    break;
                case 0xC2: case 0xC3: case 0xC5: case 0xC6: case 0xC7:
                case 0xC9: case 0xCA: case 0xCB: case 0xCD: case 0xCE: case 0xCF:
                    return fail("only baseline / extended sequential Huffman JPEG is supported");
                case 0xC4: ok = read_dht(end); break;
                case 0xDB: ok = read_dqt(end); break;
                case 0xDD: restart_interval = u16(); break;
                case 0xDA:
                    if (!frame) return fail("scan before frame");
                    ok = read_sos(end);
                    scanned = true;
                    continue;  // read_sos left pos at the next marker
                case 0xE0:
                    if (len >= 7 && std::memcmp(d + pos, "JFIF", 4) == 0) jfif = true;
                    break;
                case 0xEE:
                    if (len >= 14 && std::memcmp(d + pos, "Adobe", 5) == 0) adobe_transform = d[pos + 11];
                    break;
                default: break;
            }
            if (!ok) return false;
            pos = end;
        }
        if (!scanned) return fail("no image data");
        // colour: YCbCr unless an Adobe marker says "no transform" (libjpeg jdapimin.c default_decompress_parms)
        const bool ycc = comps.size() == 3 && !(adobe_transform == 0 && !jfif) &&
                         !(adobe_transform < 0 && !jfif && comps[0].id == 'R' && comps[1].id == 'G' && comps[2].id == 'B');
        out.width = (uint32_t)width;
        out.height = (uint32_t)height;
        out.rgb.assign((size_t)width * height * 3, 0.0f);
        // jdcolor.c build_ycc_rgb_table / ycc_rgb_convert (SCALEBITS 16)
        const int64_t ONE_HALF = (int64_t)1 << 15;
        auto FIX = [](double x) { return (int64_t)(x * 65536.0 + 0.5); };
        int cr_r[256], cb_b[256];
        int64_t cr_g[256], cb_g[256];
        for (int i = 0; i < 256; ++i) {
            const int64_t x = i - 128;
            cr_r[i] = (int)((FIX(1.40200) * x + ONE_HALF) >> 16);
            cb_b[i] = (int)((FIX(1.77200) * x + ONE_HALF) >> 16);
            cr_g[i] = -FIX(0.71414) * x;
            cb_g[i] = -FIX(0.34414) * x + ONE_HALF;
        }
        auto clamp255 = [](int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); };
        auto sample = [&](const Component& c, int xx, int yy) {  // replication upsampling
            const int sx = xx * c.h / hmax, sy = yy * c.v / vmax;
            return (int)c.samples[(size_t)sy * c.bw * 8 + sx];
        };
        for (int yy = 0; yy < height; ++yy)
            for (int xx = 0; xx < width; ++xx) {
                int r, g, b;
                if (comps.size() == 1) {
                    r = g = b = sample(comps[0], xx, yy);
                } else {
                    const int y0 = sample(comps[0], xx, yy), c1 = sample(comps[1], xx, yy),
                              c2 = sample(comps[2], xx, yy);
                    if (ycc) {
                        r = clamp255(y0 + cr_r[c2]);
                        g = clamp255(y0 + (int)((cb_g[c1] + cr_g[c2]) >> 16));
                        b = clamp255(y0 + cb_b[c1]);
                    } else {
                        r = y0;
                        g = c1;
                        b = c2;
                    }
                }
                float* o = out.rgb.data() + ((size_t)yy * width + xx) * 3;  // into_rgb32f: u8 / 255
                o[0] = (float)r / 255.0f;
                o[1] = (float)g / 255.0f;
                o[2] = (float)b / 255.0f;
            }
        return true;
    }
};

}  // namespace

bool decode_jpeg(const std::vector<uint8_t>& data, DecodedImage& out, std::string& err) {
    Decoder dec{data.data(), data.size()};
    const bool ok = dec.run(out);
    if (!ok) err = dec.err.empty() ? "corrupt JPEG" : dec.err;
    return ok;
}

}  // namespace nrt
