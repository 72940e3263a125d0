/*
 * oracle/crc32_oracle.c -- CPU ORACLE for the CRC-32 body-checksum path.
 *
 * *** TEST INFRASTRUCTURE ONLY. ***
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this file's library, and only as the checker. The product library
 * (rpc_amd/lib/librpccrc.so) never links, loads or calls it.
 *
 * What it restates
 * ----------------
 * The reference checksum is rpc_crc32() (reference crc.c:4-9, decl crc.h:8):
 *     uLong c = crc32(0L, Z_NULL, 0);  c = crc32(c, data, len);  return (uint32_t)c;
 * i.e. all arithmetic lives in the third-party system zlib, which the reference
 * does NOT vendor.  Version in the image: zlib 1.2.11
 * (Ubuntu zlib1g 1:1.2.11.dfsg-2ubuntu9.2).  Its published algorithm:
 *   * CRC-32/ISO-HDLC: reflected polynomial 0xEDB88320, register pre- and
 *     post-conditioned with 0xFFFFFFFF, bytes consumed LSB first
 *     (zlib crc32.c, "crc32_little"/byte loop; 1.2.11 uses 4-table slicing,
 *     which is an optimisation of the same byte recurrence).
 *   * crc32(crc, Z_NULL, len) returns 0 (zlib crc32.c: "if (buf == Z_NULL)
 *     return 0UL;"), so rpc_crc32(NULL, n) == 0 for every n.
 *   * The len parameter of zlib crc32() is uInt (32 bit): crc.c:7 passes a
 *     size_t which is converted modulo 2^32 (verified there:
 *     2^32+3 zero bytes give the CRC of 3 zero bytes).
 *   * crc32_combine(crc1, crc2, len2) (zlib.h:1750) -- the GF(2) shift used to
 *     define the device path's lane/chunk merges; restated with zlib 1.2.11's
 *     32x32 GF(2) matrix squaring method (gf2_matrix_times / _square).
 *   * rpc_crc32_verify (reference crc.c:11-14): equality with expected_crc.
 *
 * Everything here is the plain bit-at-a-time / byte-table form: slow on
 * purpose, obviously-correct, independent of the device kernels' tables.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define ORACLE_POLY 0xEDB88320u

/* One reflected CRC step per bit (zlib make_crc_table recurrence). */
static uint32_t oracle_byte_table[256];
static int oracle_table_ready = 0;

static void oracle_make_table(void)
{
    for (uint32_t n = 0; n < 256; n++) {
        uint32_t c = n;
        for (int k = 0; k < 8; k++)
            c = (c & 1u) ? (c >> 1) ^ ORACLE_POLY : c >> 1;
        oracle_byte_table[n] = c;
    }
    oracle_table_ready = 1;
}

/* zlib 1.2.11 crc32(crc, buf, len) semantics, including Z_NULL -> 0. */
uint32_t oracle_zlib_crc32(uint32_t crc, const uint8_t *buf, uint32_t len)
{
    if (buf == NULL)
        return 0u;
    if (!oracle_table_ready)
        oracle_make_table();
    uint32_t c = crc ^ 0xFFFFFFFFu;
    for (uint32_t i = 0; i < len; i++)
        c = (c >> 8) ^ oracle_byte_table[(c ^ buf[i]) & 0xFFu];
    return c ^ 0xFFFFFFFFu;
}

/* Bit-at-a-time variant (no table at all) used to cross-check the table. */
uint32_t oracle_crc32_bitwise(const uint8_t *buf, uint64_t len)
{
    uint32_t c = 0xFFFFFFFFu;
    for (uint64_t i = 0; i < len; i++) {
        c ^= buf[i];
        for (int k = 0; k < 8; k++)
            c = (c & 1u) ? (c >> 1) ^ ORACLE_POLY : c >> 1;
    }
    return c ^ 0xFFFFFFFFu;
}

/* rpc_crc32 restated (reference crc.c:4-9): init via crc32(0,Z_NULL,0) == 0,
 * then crc32(0, data, (uInt)len). */
uint32_t oracle_rpc_crc32(const void *data, size_t len)
{
    uint32_t c = oracle_zlib_crc32(0u, NULL, 0u);
    return oracle_zlib_crc32(c, (const uint8_t *)data, (uint32_t)len);
}

/* rpc_crc32_verify restated (reference crc.c:11-14). */
int oracle_rpc_crc32_verify(const void *data, size_t len, uint32_t expected)
{
    return oracle_rpc_crc32(data, len) == expected;
}

/* ---- zlib 1.2.11 crc32_combine (GF(2) 32x32 matrix method) ---- */
static uint32_t gf2_matrix_times(const uint32_t *mat, uint32_t vec)
{
    uint32_t sum = 0;
    while (vec) {
        if (vec & 1u)
            sum ^= *mat;
        vec >>= 1;
        mat++;
    }
    return sum;
}

static void gf2_matrix_square(uint32_t *square, const uint32_t *mat)
{
    for (int n = 0; n < 32; n++)
        square[n] = gf2_matrix_times(mat, mat[n]);
}

uint32_t oracle_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2)
{
    uint32_t even[32], odd[32];
    if (len2 == 0)
        return crc1;
    odd[0] = ORACLE_POLY; /* operator for one zero bit */
    uint32_t row = 1;
    for (int n = 1; n < 32; n++) {
        odd[n] = row;
        row <<= 1;
    }
    gf2_matrix_square(even, odd); /* two zero bits */
    gf2_matrix_square(odd, even); /* four zero bits */
    do {
        gf2_matrix_square(even, odd);
        if (len2 & 1u)
            crc1 = gf2_matrix_times(even, crc1);
        len2 >>= 1;
        if (len2 == 0)
            break;
        gf2_matrix_square(odd, even);
        if (len2 & 1u)
            crc1 = gf2_matrix_times(odd, crc1);
        len2 >>= 1;
    } while (len2 != 0);
    return crc1 ^ crc2;
}

/* Batched helper: out[i] = rpc_crc32(base + offsets[i], lengths[i]). */
void oracle_crc32_batch(const uint8_t *base, const uint64_t *offsets,
                        const uint32_t *lengths, uint64_t n, uint32_t *out)
{
    for (uint64_t i = 0; i < n; i++)
        out[i] = oracle_rpc_crc32(base + offsets[i], lengths[i]);
}

/* Equal-length batch: body i at base + i*stride. */
void oracle_crc32_uniform(const uint8_t *base, uint64_t n, uint32_t len,
                          uint64_t stride, uint32_t *out)
{
    for (uint64_t i = 0; i < n; i++)
        out[i] = oracle_rpc_crc32(base + i * stride, len);
}

/* Counter-based splitmix64 byte generator shared by tests, bench and the
 * device datagen kernel: 64-bit word k of a stream with seed s is
 * mix64(s + (k+1) * 0x9E3779B97F4A7C15), stored little-endian. */
static uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void oracle_splitmix_fill(uint8_t *dst, uint64_t nbytes, uint64_t seed,
                          uint64_t word_offset)
{
    uint64_t k = word_offset;
    uint64_t i = 0;
    while (i < nbytes) {
        uint64_t w = mix64(seed + (k + 1) * 0x9E3779B97F4A7C15ull);
        for (int b = 0; b < 8 && i < nbytes; b++, i++)
            dst[i] = (uint8_t)(w >> (8 * b));
        k++;
    }
}
