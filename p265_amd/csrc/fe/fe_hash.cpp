// Decoded picture hash (H.265 D.3.19: MD5, CRC, checksum) of one 8-bit sample plane, for
// checking a decoded picture against the stream's decoded_picture_hash SEI.  The reference
// has no SEI support (nalu.py:130-131 raises) and no picture output (p265:9 "-o" unused).
#include <cstdint>
#include <cstring>

#include "../../../include/p265fe.h"

namespace {

// MD5 (RFC 1321)
struct Md5 {
    uint32_t a = 0x67452301, b = 0xefcdab89, c = 0x98badcfe, d = 0x10325476;
    uint8_t buf[64];
    uint64_t len = 0;
    static uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
    void block(const uint8_t* p) {
        static const uint32_t K[64] = {
            0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
            0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
            0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
            0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
            0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
            0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
            0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
            0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
        static const int S[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                                  5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                                  4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                                  6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
        uint32_t m[16];
        for (int i = 0; i < 16; ++i)
            m[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
                   ((uint32_t)p[4 * i + 3] << 24);
        uint32_t A = a, B = b, C = c, D = d;
        for (int i = 0; i < 64; ++i) {
            uint32_t f;
            int g;
            if (i < 16) { f = (B & C) | (~B & D); g = i; }
            else if (i < 32) { f = (D & B) | (~D & C); g = (5 * i + 1) & 15; }
            else if (i < 48) { f = B ^ C ^ D; g = (3 * i + 5) & 15; }
            else { f = C ^ (B | ~D); g = (7 * i) & 15; }
            uint32_t t = D;
            D = C;
            C = B;
            B = B + rol(A + f + K[i] + m[g], S[i]);
            A = t;
        }
        a += A; b += B; c += C; d += D;
    }
    void update(const uint8_t* p, size_t n) {
        size_t fill = len & 63;
        len += n;
        if (fill) {
            size_t take = 64 - fill < n ? 64 - fill : n;
            std::memcpy(buf + fill, p, take);
            p += take; n -= take;
            if (fill + take < 64) return;
            block(buf);
        }
        for (; n >= 64; p += 64, n -= 64) block(p);
        std::memcpy(buf, p, n);
    }
    void final(uint8_t out[16]) {
        uint64_t bits = len * 8;
        uint8_t pad = 0x80;
        update(&pad, 1);
        uint8_t z = 0;
        while ((len & 63) != 56) update(&z, 1);
        uint8_t l[8];
        for (int i = 0; i < 8; ++i) l[i] = (uint8_t)(bits >> (8 * i));
        update(l, 8);
        uint32_t v[4] = {a, b, c, d};
        for (int i = 0; i < 4; ++i)
            for (int k = 0; k < 4; ++k) out[4 * i + k] = (uint8_t)(v[i] >> (8 * k));
    }
};

}  // namespace

extern "C" int p265fe_plane_hash(const uint8_t* plane, int width, int height, int stride, int hash_type,
                                 uint8_t out[16]) {
    if (!plane || !out || width <= 0 || height <= 0 || stride < width) return P265FE_EINVAL;
    std::memset(out, 0, 16);
    if (hash_type == P265FE_HASH_MD5) {
        Md5 m;
        for (int y = 0; y < height; ++y) m.update(plane + (size_t)y * stride, (size_t)width);
        m.final(out);
    } else if (hash_type == P265FE_HASH_CRC) {
        // (D-22): bit-serial CRC-16 (0x1021), initial 0xFFFF, 16 zero bits appended; byte-table form
        static uint16_t T[256];
        static bool init = false;
        if (!init) {
            for (int h = 0; h < 256; ++h) {
                uint32_t crc = (uint32_t)h << 8;
                for (int k = 0; k < 8; ++k) {
                    uint32_t msb = (crc >> 15) & 1;
                    crc = ((crc << 1) & 0xFFFF) ^ (msb * 0x1021);
                }
                T[h] = (uint16_t)crc;
            }
            init = true;
        }
        uint32_t crc = 0xFFFF;
        for (int y = 0; y < height; ++y) {
            const uint8_t* row = plane + (size_t)y * stride;
            for (int x = 0; x < width; ++x) crc = ((((crc & 0xFF) << 8) | row[x]) ^ T[crc >> 8]) & 0xFFFF;
        }
        for (int k = 0; k < 2; ++k) crc = (((crc & 0xFF) << 8) ^ T[crc >> 8]) & 0xFFFF;
        out[0] = (uint8_t)(crc >> 8);
        out[1] = (uint8_t)crc;
    } else if (hash_type == P265FE_HASH_CHECKSUM) {
        // (D-23): sum of (sample ^ xorMask) & 0xFF, xorMask = (x & 0xFF) ^ (y & 0xFF) ^ (x >> 8) ^ (y >> 8)
        uint32_t sum = 0;
        for (int y = 0; y < height; ++y) {
            const uint8_t* row = plane + (size_t)y * stride;
            for (int x = 0; x < width; ++x) {
                uint32_t mask = (uint32_t)((x & 0xFF) ^ (y & 0xFF) ^ (x >> 8) ^ (y >> 8));
                sum += (row[x] ^ mask) & 0xFF;
            }
        }
        out[0] = (uint8_t)(sum >> 24); out[1] = (uint8_t)(sum >> 16); out[2] = (uint8_t)(sum >> 8); out[3] = (uint8_t)sum;
    } else {
        return P265FE_EINVAL;
    }
    return P265FE_OK;
}
