// gm_inet.hpp -- nginx 1.17.3's address text rules, shared by the host compiler (set_real_ip_from
// CIDRs) and the device (the client address ngx_http_realip_module takes from a request header).
//
// Restated from nginx's published behaviour (the source is not in the reference):
//   ngx_inet_addr        dotted quad; an empty octet reads 0, an octet > 255 or any other byte
//                        fails, and so does 255.255.255.255 (it equals INADDR_NONE)
//   ngx_inet6_addr       hex groups of <= 4 digits, one "::", an IPv4 tail after the last ':'
//   ngx_parse_addr_port  the address alone, else "[v6]:port" or "v4:port" split at the first ':'
//   ngx_ptocidr          addr[/bits]; host bits past the mask are cleared
//   ngx_sock_ntop        the text $remote_addr shows after the realip module replaced the
//                        connection address: a.b.c.d, or ngx_inet6_ntop (the longest run of >= 2
//                        zero groups as "::", the first on a tie; ::ffff:a.b.c.d, ::a.b.c.d forms)
// Device code calls these only for servers that configure realip (out of the route fast path).
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#endif

namespace gm {

// the client address: family 4 (b[0..3]) or 6 (b[0..15]), port 0 = none
struct InetAddr { uint32_t fam; uint8_t b[16]; uint32_t port; };

__host__ __device__ inline bool ngx_inet4(const uint8_t *p, uint32_t n, uint8_t out[4]) {
    uint32_t addr = 0, octet = 0, dots = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t c = p[i];
        if (c - '0' < 10u) {
            octet = octet * 10 + (c - '0');
            if (octet > 255) return false;
            continue;
        }
        if (c != '.') return false;
        addr = (addr << 8) + octet;
        octet = 0;
        dots++;
    }
    if (dots != 3) return false;
    addr = (addr << 8) + octet;
    if (addr == 0xFFFFFFFFu) return false;   // INADDR_NONE
    out[0] = (uint8_t)(addr >> 24); out[1] = (uint8_t)(addr >> 16); out[2] = (uint8_t)(addr >> 8); out[3] = (uint8_t)addr;
    return true;
}

__host__ __device__ inline bool ngx_inet6(const uint8_t *p, uint32_t n, uint8_t out[16]) {
    if (n == 0) return false;
    uint32_t o = 0, groups = 8, nib = 0, word = 0;
    int zero = -1;                 // byte index of the "::" gap
    const uint8_t *digit = nullptr;   // after the last ':' (an IPv4 tail starts there)
    uint32_t rest = 0;                // bytes from that ':' (inclusive) to the end
    if (p[0] == ':') { p++; n--; }
    uint32_t i = 0;
    for (; i < n; i++) {
        const uint32_t c = p[i];
        if (c == ':') {
            if (nib) {
                digit = p + i + 1; rest = n - i;
                out[o++] = (uint8_t)(word >> 8); out[o++] = (uint8_t)word;
                if (--groups) { nib = 0; word = 0; continue; }
            } else if (zero < 0) {
                digit = p + i + 1; rest = n - i;
                zero = (int)o;
                continue;
            }
            return false;
        }
        if (c == '.' && nib) {
            if (groups < 2 || !digit) return false;
            uint8_t v4[4];
            if (!ngx_inet4(digit, rest - 1, v4)) return false;
            out[o++] = v4[0]; out[o++] = v4[1];
            word = (uint32_t)v4[2] << 8 | v4[3];
            groups--;
            break;
        }
        if (++nib > 4) return false;
        if (c - '0' < 10u) { word = word * 16 + (c - '0'); continue; }
        const uint32_t l = c | 0x20;
        if (l - 'a' < 6u) { word = word * 16 + (l - 'a') + 10; continue; }
        return false;
    }
    if (nib == 0 && zero < 0) return false;
    out[o++] = (uint8_t)(word >> 8); out[o++] = (uint8_t)word;
    if (--groups) {
        if (zero < 0) return false;
        const uint32_t gap = groups * 2;   // zero bytes to insert at `zero`
        for (int s = (int)o - 1; s >= zero; s--) out[s + gap] = out[s];
        for (uint32_t z = 0; z < gap; z++) out[zero + z] = 0;
        return true;
    }
    return zero < 0;
}

// ngx_parse_addr: 4 / 6, or 0
__host__ __device__ inline uint32_t ngx_parse_addr(const uint8_t *p, uint32_t n, uint8_t b[16]) {
    if (ngx_inet4(p, n, b)) return 4;
    if (ngx_inet6(p, n, b)) return 6;
    return 0;
}

// ngx_atoi: decimal digits only, at least one; -1 otherwise
__host__ __device__ inline int64_t ngx_atoi_dec(const uint8_t *p, uint32_t n) {
    if (n == 0) return -1;
    int64_t v = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (p[i] - '0' >= 10u) return -1;
        v = v * 10 + (p[i] - '0');
        if (v > 0x7FFFFFFF) return -1;
    }
    return v;
}

__host__ __device__ inline bool ngx_parse_addr_port(const uint8_t *p, uint32_t n, InetAddr &a) {
    a.port = 0;
    a.fam = ngx_parse_addr(p, n, a.b);
    if (a.fam) return true;
    uint32_t astart = 0, alen, pstart;   // the address part and the port's first byte
    if (n && p[0] == '[') {
        uint32_t rb = 0;
        while (rb < n && p[rb] != ']') rb++;
        if (rb >= n || rb == n - 1 || p[rb + 1] != ':') return false;
        astart = 1; alen = rb - 1; pstart = rb + 2;
    } else {
        uint32_t colon = 0;
        while (colon < n && p[colon] != ':') colon++;
        if (colon >= n) return false;
        alen = colon; pstart = colon + 1;
    }
    const int64_t port = ngx_atoi_dec(p + pstart, n - pstart);
    if (port < 1 || port > 65535) return false;
    a.fam = ngx_parse_addr(p + astart, alen, a.b);
    if (!a.fam) return false;
    a.port = (uint32_t)port;
    return true;
}

__host__ __device__ inline uint32_t put_dec(uint8_t *o, uint32_t v) {
    uint8_t t[10];
    uint32_t k = 0;
    do { t[k++] = (uint8_t)('0' + v % 10); v /= 10; } while (v);
    for (uint32_t i = 0; i < k; i++) o[i] = t[k - 1 - i];
    return k;
}

// ngx_sock_ntop (no port): the text form of the address; out holds >= 46 bytes
__host__ __device__ inline uint32_t ngx_addr_text(const InetAddr &a, uint8_t *out) {
    uint32_t k = 0;
    if (a.fam == 4) {
        for (int i = 0; i < 4; i++) {
            k += put_dec(out + k, a.b[i]);
            if (i < 3) out[k++] = '.';
        }
        return k;
    }
    const uint8_t *p = a.b;
    int zero = -1, last = -1;
    uint32_t max = 1, run = 0;
    for (int i = 0; i < 16; i += 2) {
        if (p[i] || p[i + 1]) {
            if (max < run) { zero = last; max = run; }
            run = 0;
            continue;
        }
        if (run++ == 0) last = i;
    }
    if (max < run) { zero = last; max = run; }
    int end = 16;
    if (zero == 0) {
        if ((max == 5 && p[10] == 0xFF && p[11] == 0xFF) || max == 6 || (max == 7 && p[14] != 0 && p[15] != 1)) end = 12;
        out[k++] = ':';
    }
    for (int i = 0; i < end; i += 2) {
        if (i == zero) {
            out[k++] = ':';
            i += (int)(max - 1) * 2;
            continue;
        }
        const uint32_t w = (uint32_t)p[i] * 256 + p[i + 1];
        uint8_t t[4];
        uint32_t nd = 0;
        uint32_t x = w;
        do { const uint32_t d = x & 15; t[nd++] = (uint8_t)(d < 10 ? '0' + d : 'a' + d - 10); x >>= 4; } while (x);
        for (uint32_t q = 0; q < nd; q++) out[k++] = t[nd - 1 - q];
        if (i < 14) out[k++] = ':';
    }
    if (end == 12) {
        for (int i = 12; i < 16; i++) {
            k += put_dec(out + k, p[i]);
            if (i < 15) out[k++] = '.';
        }
    }
    return k;
}

// ngx_cidr_match for one entry (fam 4 / 6, network-order bytes); an IPv4-mapped IPv6 address
// matches as IPv4
__host__ __device__ inline bool cidr_match1(const InetAddr &a, uint32_t cfam, const uint8_t *addr, const uint8_t *mask) {
    uint32_t fam = a.fam;
    const uint8_t *b = a.b;
    if (fam == 6) {
        bool mapped = b[10] == 0xFF && b[11] == 0xFF;
        for (int i = 0; i < 10; i++) mapped = mapped && b[i] == 0;
        if (mapped) { fam = 4; b += 12; }
    }
    if (fam != cfam) return false;
    const uint32_t nb = fam == 4 ? 4 : 16;
    for (uint32_t i = 0; i < nb; i++) if ((b[i] & mask[i]) != addr[i]) return false;
    return true;
}

}  // namespace gm
