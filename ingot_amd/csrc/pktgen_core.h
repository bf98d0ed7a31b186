// pktgen_core.h — the synthetic traffic generator shared by the device
// (pktgen.hip, ingot_pktgen_fill) and the host (pktgen_host.cpp,
// ingot_pktgen_fill_host, built with g++ for bench.py's CPU baseline, which
// runs before the process touches the GPU).  Every frame is a pure function
// of (profile, seed, index): `plan()` draws the header chain and the length
// from a counter-based SplitMix64 stream, `write_frame()` lays the bytes
// down (clipped to the frame length).  Bench/test infrastructure, not the
// parse path.
#pragma once

#include <math.h>
#include <stdint.h>

#include "../../include/ingot_pktgen.h"

#if defined(__HIP__)
#define INGOT_HD __host__ __device__
#else
#define INGOT_HD
#endif

namespace ingot_pktgen {

struct Rng {
    uint64_t s;
    INGOT_HD explicit Rng(uint64_t seed, uint64_t idx, uint64_t stream = 0) {
        s = seed * 0x9E3779B97F4A7C15ull ^ (idx + 0x632BE59BD9B4E019ull) * 0xD1B54A32D192ED03ull ^
            stream * 0x8CB92BA72F3D8DD7ull;
        next();
    }
    INGOT_HD uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    INGOT_HD uint32_t u32() { return (uint32_t)(next() >> 32); }
    INGOT_HD uint32_t range(uint32_t lo, uint32_t hi) {  // inclusive
        return lo + (uint32_t)(((next() >> 32) * (uint64_t)(hi - lo + 1)) >> 32);
    }
    INGOT_HD bool chance(uint32_t permille) { return range(0, 999) < permille; }
    INGOT_HD double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

struct Plan {
    uint32_t len;
    uint32_t n_vlan;
    uint32_t tpid[2];
    uint32_t ethertype;  // after tags
    uint32_t ihl;
    uint32_t n_eh;
    uint32_t eh_type[4];
    uint32_t eh_ext[4];
    uint32_t proto;  // L4 protocol (the last next_header)
    uint32_t doff;
    uint32_t flow;   // 0 = none, else 1..FLOWS_N
    uint32_t hdr_len;
    // Geneve tunnel profiles: the fields above describe the inner frame,
    // which starts at inner_off; these describe the outer layers.
    uint32_t tun;
    uint32_t inner_off;
    uint32_t o_et;        // outer ethertype
    uint32_t o_ihl;       // outer IPv4 (adversarial)
    uint32_t o_n_eh;
    uint32_t o_eh_type[3];
    uint32_t o_eh_ext[3];
    uint32_t o_proto;     // outer L4 protocol
    uint32_t o_doff;
    uint32_t g_words;     // Geneve opt_len
    uint32_t g_n_opt;     // well-formed options (g_rand = 0)
    uint32_t g_len[3];    // option data words
    uint32_t g_rand;      // 1: the options span is random bytes
};

// Zipf(s) over {1..n} by rejection-inversion (Hörmann & Derflinger 1996).
struct Zipf {
    double s, n;
    INGOT_HD double h(double x) const { return exp(-s * log(x)); }
    INGOT_HD static double helper1(double x) { return fabs(x) > 1e-8 ? log1p(x) / x : 1 - x * (0.5 - x * (1.0 / 3.0 - 0.25 * x)); }
    INGOT_HD static double helper2(double x) { return fabs(x) > 1e-8 ? expm1(x) / x : 1 + x * 0.5 * (1 + x * (1.0 / 3.0) * (1 + 0.25 * x)); }
    INGOT_HD double hint(double x) const { const double lx = log(x); return helper2((1 - s) * lx) * lx; }
    INGOT_HD double hinv(double x) const {
        double t = x * (1 - s);
        if (t < -1) t = -1;
        return exp(helper1(t) * x);
    }
    INGOT_HD uint32_t sample(Rng& r) const {
        const double hx1 = hint(1.5) - 1.0, hn = hint(n + 0.5);
        const double sv = 2.0 - hinv(hint(2.5) - h(2.0));
        for (int it = 0; it < 64; ++it) {
            const double u = hn + r.unit() * (hx1 - hn);
            const double x = hinv(u);
            double k = floor(x + 0.5);
            if (k < 1) k = 1;
            if (k > n) k = n;
            if (k - x <= sv || u >= hint(k + 0.5) - h(k)) return (uint32_t)k;
        }
        return 1;
    }
};

constexpr uint32_t EH_CHOICES_C3[4] = {0, 60, 43, 44};

INGOT_HD inline uint32_t eh_len(uint32_t type, uint32_t ext) { return type == 44 ? 8u : 8u + 8u * ext; }

// Random chain from the Ethernet header at `hdr - 14`; everything the parser
// must reject appears.  Returns the header bytes through L4.
INGOT_HD inline uint32_t plan_adversarial_chain(Rng& r, Plan& p, uint32_t hdr) {
    const uint32_t ets[8] = {0x0800, 0x86dd, 0x8100, 0x9100, 0x0806, 0x0800, 0x86dd, 0};
    uint32_t et = ets[r.range(0, 7)];
    if (et == 0) et = r.range(0, 0xffff);
    p.n_vlan = 0;
    while ((et == 0x8100 || et == 0x9100) && p.n_vlan < 2) {
        p.tpid[p.n_vlan++] = et;
        hdr += 4;
        const uint32_t nx[5] = {0x0800, 0x86dd, 0x8100, 0x9100, 0x0806};
        et = nx[r.range(0, 4)];
    }
    // a third TPID stays as the inner ethertype (L3 choice -> Unwanted)
    p.ethertype = et;
    const uint32_t protos[12] = {6, 17, 1, 58, 0, 43, 44, 60, 59, 253, 135, 50};
    if (et == 0x0800) {
        p.ihl = r.chance(600) ? 5 : r.range(0, 15);
        hdr += (p.ihl * 4 > 20 ? p.ihl * 4 : 20);
        p.proto = r.chance(900) ? protos[r.range(0, 11)] : r.range(0, 255);
    } else if (et == 0x86dd) {
        hdr += 40;
        p.n_eh = r.chance(500) ? 0 : r.range(1, 4);
        const uint32_t ehs[10] = {0, 43, 44, 60, 135, 139, 140, 253, 254, 44};
        for (uint32_t k = 0; k < p.n_eh; ++k) {
            p.eh_type[k] = ehs[r.range(0, 9)];
            p.eh_ext[k] = r.chance(700) ? r.range(0, 2) : r.range(0, 255);
            hdr += eh_len(p.eh_type[k], p.eh_ext[k]);
        }
        p.proto = r.chance(900) ? protos[r.range(0, 11)] : r.range(0, 255);
    }
    if (p.proto == 6) {
        p.doff = r.chance(600) ? 5 : r.range(0, 15);
        hdr += (p.doff * 4 > 20 ? p.doff * 4 : 20);
    } else {
        hdr += 8;
    }
    return hdr;
}

// Lengths cluster around the chain's end so every truncation point is hit.
INGOT_HD inline uint32_t adversarial_len(Rng& r, uint32_t hdr, uint32_t wide) {
    const uint32_t mode = r.range(0, 9);
    uint32_t len;
    if (mode < 4) len = hdr + r.range(0, 32);
    else if (mode < 8) len = r.range(0, hdr + 8);
    else len = r.range(0, wide);
    return len > 65535u ? 65535u : len;
}

// GeneveOverV6Tunnel traffic (OPTE's inbound path, ingot-examples/src/
// packets.rs:27-40).  Realistic: outer Eth / IPv6 (HBH p .05) / UDP 6081 /
// Geneve opt_len 0 (p .1), 1 = one 4-B option class 0x0129 (p .8), or 3 = that
// + one option with 4 B of data (p .1); inner Eth with ARP p .02, IPv4 p .68
// (ihl 5 p .95), IPv6 p .30 (one fragment EH p .05); TCP p .75 (data_offset 8
// p .6, 5 p .3, else U[6,15]), UDP p .22, ICMP p .03; inner frame length
// U[64,1500] raised to fit.  Adversarial: outer ethertype / EH chain / L4
// protocol / option spans perturbed, the inner chain from the adversarial
// planner, lengths clustered at the chain's end.
INGOT_HD inline Plan plan_geneve(bool adv, Rng& r) {
    Plan p{};
    p.tun = 1;
    uint32_t hdr = 14;
    p.o_et = 0x86dd;
    if (adv) {
        const uint32_t u = r.range(0, 9);
        p.o_et = u < 8 ? 0x86dd : u == 8 ? 0x0800 : r.range(0, 0xffff);
    }
    p.o_proto = 17;
    if (p.o_et == 0x86dd) {
        hdr += 40;
        p.o_n_eh = adv ? (r.chance(700) ? 0 : r.range(1, 3)) : (r.chance(50) ? 1 : 0);
        const uint32_t ehs[6] = {0, 60, 43, 44, 135, 253};
        for (uint32_t k = 0; k < p.o_n_eh; ++k) {
            p.o_eh_type[k] = adv ? ehs[r.range(0, 5)] : 0;
            p.o_eh_ext[k] = adv ? (r.chance(800) ? r.range(0, 2) : r.range(0, 255)) : 0;
            hdr += eh_len(p.o_eh_type[k], p.o_eh_ext[k]);
        }
    } else if (p.o_et == 0x0800) {
        p.o_ihl = r.chance(700) ? 5 : r.range(0, 15);
        hdr += p.o_ihl * 4 > 20 ? p.o_ihl * 4 : 20;
    }
    if (adv && !r.chance(850)) {
        const uint32_t ps[5] = {6, 1, 58, 50, 0};
        p.o_proto = ps[r.range(0, 4)];
        if (p.o_proto == 0 && p.o_et != 0x86dd) p.o_proto = r.range(0, 255);
    }
    if (p.o_proto == 6) {
        p.o_doff = r.chance(600) ? 5 : r.range(0, 15);
        hdr += p.o_doff * 4 > 20 ? p.o_doff * 4 : 20;
    } else {
        hdr += 8;
    }
    // Geneve
    if (adv && r.chance(400)) {
        p.g_rand = 1;
        p.g_words = r.range(0, 63);
    } else {
        const uint32_t u = r.range(0, 9);
        if (u == 0) {
            p.g_n_opt = 0;
        } else if (u < 9) {
            p.g_n_opt = 1;
            p.g_len[0] = 0;
        } else {
            p.g_n_opt = 2;
            p.g_len[0] = 0;
            p.g_len[1] = adv ? r.range(0, 3) : 1;
        }
        for (uint32_t k = 0; k < p.g_n_opt; ++k) p.g_words += 1 + p.g_len[k];
    }
    hdr += 8 + 4 * p.g_words;
    p.inner_off = hdr;
    hdr += 14;
    if (adv) {
        hdr = plan_adversarial_chain(r, p, hdr);
        p.hdr_len = hdr;
        p.len = adversarial_len(r, hdr, hdr + 64);
        return p;
    }
    const uint32_t u = r.range(0, 99);
    p.ethertype = u < 2 ? 0x0806 : u < 70 ? 0x0800 : 0x86dd;
    if (p.ethertype == 0x0800) {
        p.ihl = r.chance(950) ? 5 : r.range(6, 8);
        hdr += p.ihl * 4;
    } else if (p.ethertype == 0x86dd) {
        hdr += 40;
        p.n_eh = r.chance(50) ? 1 : 0;
        p.eh_type[0] = 44;
        if (p.n_eh) hdr += 8;
    }
    if (p.ethertype != 0x0806) {
        const uint32_t l4 = r.range(0, 99);
        if (l4 < 75) {
            p.proto = 6;
            const uint32_t d = r.range(0, 9);
            p.doff = d < 6 ? 8 : d < 9 ? 5 : r.range(6, 15);
            hdr += p.doff * 4;
        } else if (l4 < 97) {
            p.proto = 17;
            hdr += 8;
        } else {
            p.proto = p.ethertype == 0x0800 ? 1 : 58;
            hdr += 8;
        }
    }
    p.hdr_len = hdr;
    const uint32_t inner_len = r.range(64, 1500);
    p.len = p.inner_off + inner_len < hdr ? hdr : p.inner_off + inner_len;
    return p;
}

INGOT_HD inline Plan plan(int profile, uint64_t seed, uint64_t i) {
    Rng r(seed, i);
    Plan p{};
    uint32_t hdr = 14;
    if (profile == INGOT_GEN_V4UDP64) {
        p.len = 64;
        p.ethertype = 0x0800;
        p.ihl = 5;
        p.proto = 17;
        p.hdr_len = 42;
        return p;
    }
    if (profile == INGOT_GEN_ADVERSARIAL) {
        hdr = plan_adversarial_chain(r, p, hdr);
        p.hdr_len = hdr;
        p.len = adversarial_len(r, hdr, 160);
        return p;
    }
    if (profile == INGOT_GEN_GENEVE || profile == INGOT_GEN_GENEVE_ADVERSARIAL) {
        return plan_geneve(profile == INGOT_GEN_GENEVE_ADVERSARIAL, r);
    }

    // MIXED / VLAN_V6EH / FLOWS
    const bool c4 = profile != INGOT_GEN_MIXED;
    if (c4 && r.chance(500)) {
        if (r.chance(200)) {
            p.n_vlan = 2;
            p.tpid[0] = 0x9100;
            p.tpid[1] = 0x8100;
        } else {
            p.n_vlan = 1;
            p.tpid[0] = 0x8100;
        }
        hdr += 4 * p.n_vlan;
    }
    bool v6 = r.chance(500);
    bool tcp = r.chance(500);
    if (profile == INGOT_GEN_FLOWS) {
        const Zipf z{1.1, (double)INGOT_GEN_FLOWS_N};
        p.flow = z.sample(r);
        Rng fr(seed ^ 0xF10Full, p.flow);
        v6 = fr.chance(500);
        tcp = fr.chance(500);
    }
    p.ethertype = v6 ? 0x86dd : 0x0800;
    if (!v6) {
        p.ihl = r.chance(900) ? 5 : r.range(6, 15);
        hdr += p.ihl * 4;
    } else {
        hdr += 40;
        const bool want_eh = c4 ? r.chance(500) : r.chance(200);
        p.n_eh = want_eh ? r.range(1, 3) : 0;
        for (uint32_t k = 0; k < p.n_eh; ++k) {
            p.eh_type[k] = EH_CHOICES_C3[r.range(0, 3)];
            p.eh_ext[k] = r.range(0, 3);
            hdr += eh_len(p.eh_type[k], p.eh_ext[k]);
        }
    }
    p.proto = tcp ? 6 : 17;
    if (tcp) {
        p.doff = r.chance(700) ? 5 : r.range(6, 15);
        hdr += p.doff * 4;
    } else {
        hdr += 8;
    }
    p.hdr_len = hdr;
    uint32_t len = r.range(64, 1500);
    p.len = len < hdr ? hdr : len;
    return p;
}

struct Writer {
    uint8_t* f;
    uint32_t len;
    INGOT_HD void u8(uint32_t at, uint32_t v) const {
        if (at < len) f[at] = (uint8_t)v;
    }
    INGOT_HD void u16(uint32_t at, uint32_t v) const { u8(at, v >> 8); u8(at + 1, v); }
    INGOT_HD void u32(uint32_t at, uint32_t v) const { u16(at, v >> 16); u16(at + 2, v); }
    INGOT_HD void rnd(uint32_t at, uint32_t n, Rng& r) const {
        for (uint32_t k = 0; k < n; k += 4) {
            const uint32_t v = r.u32();
            for (uint32_t j = 0; j < 4 && k + j < n; ++j) u8(at + k + j, v >> (24 - 8 * j));
        }
    }
};

// The Ethernet -> (VLAN) -> L3 -> L4 chain of `p`, Ethernet at frame offset
// `o` (0, or the tunnel's inner_off).
INGOT_HD inline void write_chain(int profile, const Plan& p, const Writer& w, Rng& r, Rng& tuple,
                            uint32_t o) {
    const uint32_t len = w.len;
    const bool adv = profile == INGOT_GEN_ADVERSARIAL || profile == INGOT_GEN_GENEVE_ADVERSARIAL;
    // Ethernet
    if (profile == INGOT_GEN_V4UDP64) {
        for (uint32_t k = 0; k < 6; ++k) w.u8(k, 0x00), w.u8(6 + k, 0xff);
    } else {
        w.rnd(o, 12, r);
    }
    w.u16(o + 12, p.n_vlan ? p.tpid[0] : p.ethertype);
    o += 14;
    for (uint32_t v = 0; v < p.n_vlan; ++v) {
        w.u16(o, r.u32());  // TCI
        const uint32_t next = v + 1 < p.n_vlan ? p.tpid[v + 1] : p.ethertype;
        w.u16(o + 2, next);
        o += 4;
    }
    const uint32_t l3 = o;
    if (p.ethertype == 0x0800) {
        if (profile == INGOT_GEN_V4UDP64) {
            w.u8(o, 0x45); w.u8(o + 1, 0); w.u16(o + 2, 50); w.u32(o + 4, 0);
            w.u8(o + 8, 0xf0); w.u8(o + 9, 17); w.u16(o + 10, 0);
            w.u32(o + 12, r.u32()); w.u32(o + 16, r.u32());
            o += 20;
            w.u16(o, r.u32()); w.u16(o + 2, r.u32()); w.u16(o + 4, 30); w.u16(o + 6, 0);
            for (uint32_t k = 0; k < 8; ++k) w.u8(o + 8 + k, k);  // bench body 0..7
            return;
        }
        const uint32_t hl = p.ihl * 4 > 20 ? p.ihl * 4 : 20;
        w.u8(o, 0x40 | p.ihl);
        w.u8(o + 1, r.u32());
        w.u16(o + 2, len > l3 ? len - l3 : 0);
        w.u16(o + 4, r.u32());
        w.u16(o + 6, adv ? r.u32() : 0x4000);
        w.u8(o + 8, r.range(1, 255));
        w.u8(o + 9, p.proto);
        w.u16(o + 10, r.u32());
        w.u32(o + 12, tuple.u32());
        w.u32(o + 16, tuple.u32());
        if (hl > 20) w.rnd(o + 20, hl - 20, r);
        o += hl;
    } else if (p.ethertype == 0x86dd) {
        w.u32(o, 0x60000000u | (r.u32() & 0x0fffffffu));
        w.u16(o + 4, len > l3 + 40 ? len - l3 - 40 : 0);
        w.u8(o + 6, p.n_eh ? p.eh_type[0] : p.proto);
        w.u8(o + 7, r.range(1, 255));
        for (uint32_t k = 0; k < 8; ++k) w.u32(o + 8 + 4 * k, tuple.u32());
        o += 40;
        for (uint32_t k = 0; k < p.n_eh; ++k) {
            const uint32_t nh = k + 1 < p.n_eh ? p.eh_type[k + 1] : p.proto;
            w.u8(o, nh);
            if (p.eh_type[k] == 44) {
                w.u8(o + 1, adv ? r.u32() : 0);
                w.u16(o + 2, r.u32());
                w.u32(o + 4, r.u32());
                o += 8;
            } else {
                w.u8(o + 1, p.eh_ext[k]);
                w.rnd(o + 2, 6 + 8 * p.eh_ext[k], r);
                o += 8 + 8 * p.eh_ext[k];
            }
        }
    } else {
        return;  // unknown ethertype / ARP: the rest stays pattern
    }
    // L4
    const uint32_t sport = tuple.u32() & 0xffffu, dport = tuple.u32() & 0xffffu;
    if (p.proto == 6) {
        const uint32_t hl = p.doff * 4 > 20 ? p.doff * 4 : 20;
        w.u16(o, sport); w.u16(o + 2, dport);
        w.u32(o + 4, r.u32()); w.u32(o + 8, r.u32());
        w.u8(o + 12, (p.doff << 4) | (adv ? (r.u32() & 0xf) : 0));
        w.u8(o + 13, r.u32());
        w.u16(o + 14, r.u32()); w.u16(o + 16, r.u32()); w.u16(o + 18, r.u32());
        if (hl > 20) w.rnd(o + 20, hl - 20, r);
    } else if (p.proto == 17) {
        w.u16(o, sport); w.u16(o + 2, dport);
        w.u16(o + 4, len > o ? len - o : 0);
        w.u16(o + 6, r.u32());
    } else {
        w.rnd(o, 8, r);
    }
}

// Outer Ethernet / IPv6 (or the adversarial IPv4 / other) / UDP (or TCP) /
// Geneve + options of a tunnel frame.
INGOT_HD inline void write_outer(const Plan& p, const Writer& w, Rng& r) {
    const uint32_t len = w.len;
    w.rnd(0, 12, r);
    w.u16(12, p.o_et);
    uint32_t o = 14;
    if (p.o_et == 0x86dd) {
        w.u32(o, 0x60000000u | (r.u32() & 0x000fffffu));
        w.u16(o + 4, len > o + 40 ? len - o - 40 : 0);
        w.u8(o + 6, p.o_n_eh ? p.o_eh_type[0] : p.o_proto);
        w.u8(o + 7, 255);
        w.u8(o + 8, 0xfd);  // ULA fd00::/8 underlay
        w.rnd(o + 9, 7, r);
        w.u8(o + 24, 0xfd);
        w.rnd(o + 25, 15, r);
        w.rnd(o + 16, 8, r);
        o += 40;
        for (uint32_t k = 0; k < p.o_n_eh; ++k) {
            const uint32_t nh = k + 1 < p.o_n_eh ? p.o_eh_type[k + 1] : p.o_proto;
            w.u8(o, nh);
            if (p.o_eh_type[k] == 44) {
                w.u8(o + 1, 0);
                w.u16(o + 2, r.u32());
                w.u32(o + 4, r.u32());
                o += 8;
            } else {
                w.u8(o + 1, p.o_eh_ext[k]);
                w.rnd(o + 2, 6 + 8 * p.o_eh_ext[k], r);
                o += 8 + 8 * p.o_eh_ext[k];
            }
        }
    } else if (p.o_et == 0x0800) {
        const uint32_t hl = p.o_ihl * 4 > 20 ? p.o_ihl * 4 : 20;
        w.u8(o, 0x40 | p.o_ihl);
        w.rnd(o + 1, 8, r);
        w.u8(o + 9, p.o_proto);
        w.rnd(o + 10, hl - 10, r);
        o += hl;
    } else {
        return;
    }
    if (p.o_proto == 6) {
        const uint32_t hl = p.o_doff * 4 > 20 ? p.o_doff * 4 : 20;
        w.rnd(o, 12, r);
        w.u8(o + 12, p.o_doff << 4);
        w.rnd(o + 13, hl - 13, r);
        o += hl;
    } else if (p.o_proto == 17) {
        w.u16(o, 0xc000u | (r.u32() & 0x3fffu));  // flow-entropy source port
        w.u16(o + 2, 6081);                       // Geneve (RFC 8926)
        w.u16(o + 4, len > o ? len - o : 0);
        w.u16(o + 6, 0);
        o += 8;
    } else {
        w.rnd(o, 8, r);
        o += 8;
    }
    // Geneve
    w.u8(o, p.g_words & 0x3fu);   // version 0 | opt_len
    w.u8(o + 1, 0);               // flags
    w.u16(o + 2, 0x6558);         // Transparent Ethernet Bridging
    w.u32(o + 4, r.u32() & 0xffffff00u);  // vni | reserved 0
    o += 8;
    if (p.g_rand) {
        w.rnd(o, 4 * p.g_words, r);
        return;
    }
    for (uint32_t k = 0; k < p.g_n_opt; ++k) {
        const bool oxide = k == 0;
        w.u16(o, oxide ? 0x0129 : 0x0102);
        w.u8(o + 2, oxide ? 0 : (r.u32() & 0x7fu));
        w.u8(o + 3, p.g_len[k]);
        w.rnd(o + 4, 4 * p.g_len[k], r);
        o += 4 + 4 * p.g_len[k];
    }
}

INGOT_HD inline void write_frame(int profile, uint64_t seed, uint64_t i, const Plan& p, uint8_t* f,
                            uint32_t len) {
    Rng r(seed, i, 1);
    Rng fr(seed ^ 0xF10Full, p.flow, 1);  // per-flow tuple (FLOWS)
    Rng& tuple = p.flow ? fr : r;
    const Writer w{f, len};
    if (p.tun) write_outer(p, w, r);
    write_chain(profile, p, w, r, tuple, p.tun ? p.inner_off : 0u);
}


// Word w (16 B) of the pattern fill under the frames: adversarial profiles
// get random bytes (so unknown fields are arbitrary), the rest a cheap
// counter pattern.  Bytes past the last whole word: (t * 13 + 7).
INGOT_HD inline void pattern_word(int profile, uint64_t seed, uint64_t w, uint32_t v[4]) {
    if (profile == INGOT_GEN_ADVERSARIAL || profile == INGOT_GEN_GENEVE_ADVERSARIAL) {
        Rng r(seed ^ 0xA5A5ull, w, 7);
        const uint64_t a = r.next(), b = r.next();
        v[0] = (uint32_t)a;
        v[1] = (uint32_t)(a >> 32);
        v[2] = (uint32_t)b;
        v[3] = (uint32_t)(b >> 32);
    } else {
        const uint32_t x = (uint32_t)(w * 0x01010101u);
        v[0] = x;
        v[1] = x + 0x04040404u;
        v[2] = x + 0x08080808u;
        v[3] = x + 0x0c0c0c0cu;
    }
}

}  // namespace ingot_pktgen
