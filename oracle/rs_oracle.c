/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.
 *
 * A faithful scalar C restatement of slime's internal/rs and internal/rs/gf
 * (reference: /root/reference, encryptio/slime @ v0). It is the CHECKER for
 * the HIP path and the "port" CPU baseline in bench.py. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product library (slime_amd/lib/libslime_rs.so) never links or calls it.
 *
 * Parity pinning: this restatement is checked against every known-answer test
 * the reference's own test files hold (tests/golden/reference_kats.json,
 * extracted by tests/golden/make_kats.py from internal/rs/{matrix,vector}_test.go and
 * internal/rs/gf/{gf,map}_test.go) and against an independent Python big-int
 * restatement (oracle/oracle_py.py). The reference is Go and no Go toolchain
 * exists in this image, so there is no oracle/_ref build.
 *
 * Arithmetic is deliberately the reference's own: uint64 products and `%`
 * twice per term, one output row at a time (internal/rs/vector.go:90-102).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define GF_P 4294967291ull /* internal/rs/gf/map.go:7  MaxVal = 1<<32 - 5 */

/* Status codes mirror include/slime_rs.h so tests can compare error paths. */
enum {
    OR_OK = 0,
    OR_VARYING_LENGTH = 1,   /* vector.go:21 */
    OR_LEN_MISMATCH = 2,     /* vector.go:52 */
    OR_EMPTY = 3,            /* vector.go:56 */
    OR_NO_INDICES = 4,       /* vector.go:66 */
    OR_NONZERO = 5,          /* matrix.go:68 */
    OR_ONE = 6,              /* matrix.go:77 */
    OR_ZERO = 7,             /* matrix.go:92 */
    OR_INDEX_RANGE = 8,      /* Go index-out-of-range panic */
    OR_MAPPING_FALLBACK = 12 /* map.go:64-66 random fallback needed */
};

/* internal/rs/gf/gf.go:5-44 — fixed square-and-multiply chain for x^(p-2). */
uint32_t oracle_gf_minverse(uint32_t in) {
    uint64_t n = in;
    uint64_t o = (((n * n) % GF_P) * n) % GF_P;
    for (int i = 0; i < 27; i++) o = (((o * o) % GF_P) * n) % GF_P;
    o = (o * o) % GF_P;
    o = (o * o) % GF_P;
    o = (((o * o) % GF_P) * n) % GF_P;
    return (uint32_t)o;
}

/* internal/rs/gf/gf.go:46-60 — recursive power. */
uint32_t oracle_gf_raise(uint32_t x, uint32_t n) {
    if (n == 0) return 1;
    if (x == 0 || x == 1) return x;
    uint32_t v = oracle_gf_raise((uint32_t)(((uint64_t)x * x) % GF_P), n / 2);
    if (n % 2 == 1) v = (uint32_t)(((uint64_t)x * v) % GF_P);
    return v;
}

/* internal/rs/matrix.go:8-22 — (d+p) x d, m[i][j] = Raise(j+1, i). */
void oracle_vandermonde(int d, int p, uint32_t *m) {
    for (int i = 0; i < d + p; i++)
        for (int j = 0; j < d; j++) m[(size_t)i * d + j] = oracle_gf_raise((uint32_t)(j + 1), (uint32_t)i);
}

/* internal/rs/matrix.go:35-97 — Gauss-Jordan on columns of a rows x cols matrix. */
int oracle_solve_sub_identity(uint32_t *m, int rows, int cols) {
#define M(r, c) m[(size_t)(r) * cols + (c)]
    for (int i = 0; i < cols; i++) {
        if (M(i, i) == 0) {
            for (int j = i + 1; j < cols; j++) {
                if (M(i, j) != 0) {
                    for (int r = 0; r < rows; r++) { uint32_t t = M(r, i); M(r, i) = M(r, j); M(r, j) = t; }
                    break;
                }
            }
            if (M(i, i) == 0) return OR_NONZERO;
        }
        if (M(i, i) != 1) {
            uint32_t n = oracle_gf_minverse(M(i, i));
            for (int r = 0; r < rows; r++) M(r, i) = (uint32_t)(((uint64_t)M(r, i) * n) % GF_P);
            if (M(i, i) != 1) return OR_ONE;
        }
        for (int j = 0; j < cols; j++) {
            if (j == i) continue;
            if (M(i, j) != 0) {
                uint32_t n = (uint32_t)(GF_P - M(i, j));
                for (int r = 0; r < rows; r++) {
                    uint64_t val = ((uint64_t)M(r, i) * n) % GF_P;
                    M(r, j) = (uint32_t)(((uint64_t)M(r, j) + val) % GF_P);
                }
                if (M(i, j) != 0) return OR_ZERO;
            }
        }
    }
    return OR_OK;
#undef M
}

/* internal/rs/matrix.go:27-31 */
int oracle_parity_matrix(int d, int p, uint32_t *m) {
    oracle_vandermonde(d, p, m);
    return oracle_solve_sub_identity(m, d + p, d);
}

/* internal/rs/matrix.go:112-121 — column-reduce [m; I], return the bottom d rows. */
int oracle_invert_matrix(const uint32_t *m, int d, uint32_t *inv) {
    uint32_t *c = (uint32_t *)calloc((size_t)2 * d * d, sizeof(uint32_t));
    if (!c) return -1;
    memcpy(c, m, (size_t)d * d * sizeof(uint32_t));
    for (int i = 0; i < d; i++) c[(size_t)(d + i) * d + i] = 1;
    int st = oracle_solve_sub_identity(c, 2 * d, d);
    if (st == OR_OK) memcpy(inv, c + (size_t)d * d, (size_t)d * d * sizeof(uint32_t));
    free(c);
    return st;
}

/* internal/rs/vector.go:90-102 — the reference's data path, verbatim arithmetic. */
void oracle_apply_matrix(const uint32_t *mat, int rows, int k, const uint32_t *const *in, uint32_t *const *out,
                         uint64_t len) {
    for (int i = 0; i < rows; i++) {
        const uint32_t *row = mat + (size_t)i * k;
        for (uint64_t b = 0; b < len; b++) {
            uint64_t o = 0;
            for (int j = 0; j < k; j++) o = (((uint64_t)in[j][b] * (uint64_t)row[j]) % GF_P + o) % GF_P;
            out[i][b] = (uint32_t)o;
        }
    }
}

/* internal/rs/vector.go:18-41 (the matrix cache of matrixcache.go is replaced by a fresh build). */
int oracle_create_parity(const uint32_t *const *data, const uint64_t *lens, int ndata, int index, uint32_t *out) {
    for (int i = 1; i < ndata; i++)
        if (lens[i] != lens[0]) return OR_VARYING_LENGTH;
    if (ndata <= 0) return OR_INDEX_RANGE; /* Go: data[0] on an empty slice */
    int p = index >= ndata ? index - ndata + 1 : 0;
    if (index < 0) return OR_INDEX_RANGE;
    uint32_t *m = (uint32_t *)malloc((size_t)(ndata + p) * ndata * sizeof(uint32_t));
    if (!m) return -1;
    int st = oracle_parity_matrix(ndata, p, m);
    if (st == OR_OK) oracle_apply_matrix(m + (size_t)index * ndata, 1, ndata, data, &out, lens[0]);
    free(m);
    return st;
}

/* internal/rs/vector.go:50-88 — recomputes all k data rows through applyMatrix. */
int oracle_recover_data(const uint32_t *const *chunks, const uint64_t *lens, const int *indices, int nchunks,
                        int nindices, uint32_t *const *out) {
    if (nchunks != nindices) return OR_LEN_MISMATCH;
    if (nchunks == 0) return OR_EMPTY;
    int maxIndex = -1;
    for (int i = 0; i < nindices; i++)
        if (indices[i] > maxIndex) maxIndex = indices[i];
    if (maxIndex == -1) return OR_NO_INDICES;
    for (int i = 0; i < nindices; i++)
        if (indices[i] < 0) return OR_INDEX_RANGE;
    int d = nchunks;
    uint32_t *m = (uint32_t *)malloc((size_t)(d + maxIndex) * d * sizeof(uint32_t));
    uint32_t *have = (uint32_t *)malloc((size_t)d * d * sizeof(uint32_t));
    uint32_t *inv = (uint32_t *)malloc((size_t)d * d * sizeof(uint32_t));
    int st = (m && have && inv) ? oracle_parity_matrix(d, maxIndex, m) : -1;
    if (st == OR_OK) {
        for (int i = 0; i < d; i++) memcpy(have + (size_t)i * d, m + (size_t)indices[i] * d, d * sizeof(uint32_t));
        st = oracle_invert_matrix(have, d, inv);
    }
    if (st == OR_OK) {
        /* applyMatrix indexes in[j][b] for b < len(out[i]) = len(chunks[0]) */
        for (int i = 1; i < d; i++)
            if (lens[i] < lens[0]) { st = OR_INDEX_RANGE; break; }
    }
    if (st == OR_OK) oracle_apply_matrix(inv, d, d, chunks, out, lens[0]);
    free(m);
    free(have);
    free(inv);
    return st;
}

/* internal/rs/gf/map.go:74-98 and :15-33 — big-endian packing, zero low bytes in a partial last word. */
static void pack_be(const uint8_t *in, uint64_t len, uint32_t *out) {
    uint64_t full = len / 4;
    for (uint64_t i = 0; i < full; i++)
        out[i] = ((uint32_t)in[i * 4] << 24) | ((uint32_t)in[i * 4 + 1] << 16) | ((uint32_t)in[i * 4 + 2] << 8) |
                 (uint32_t)in[i * 4 + 3];
    uint64_t extra = len - full * 4;
    if (extra) {
        uint32_t w = 0;
        for (uint64_t i = 0; i < extra; i++) w += (uint32_t)in[full * 4 + i] << ((3 - i) * 8);
        out[full] = w;
    }
}

void oracle_map_to_gf_with(const uint8_t *in, uint64_t len, uint32_t n, uint32_t *out) {
    pack_be(in, len, out);
    for (uint64_t i = 0; i < (len + 3) / 4; i++) out[i] ^= n;
}

/*
 * internal/rs/gf/map.go:15-67. The deterministic part (mapping 0, then 1<<31)
 * is restated exactly. The reference's rand.Uint32() fallback is not
 * reproducible; here it draws candidates from `cands` in order (the caller's
 * stream) and returns OR_MAPPING_FALLBACK if none of them fits.
 */
int oracle_map_to_gf(const uint8_t *in, uint64_t len, const uint32_t *cands, int ncands, uint32_t *mapping,
                     uint32_t *out) {
    uint64_t nw = (len + 3) / 4;
    pack_be(in, len, out);
    int zero_ok = 1;
    for (uint64_t i = 0; i < nw; i++)
        if (out[i] >= GF_P) { zero_ok = 0; break; }
    if (zero_ok) { *mapping = 0; return OR_OK; }
    uint32_t outn = 1u << 31;
    int ci = 0;
    for (;;) {
        int ok = 1;
        for (uint64_t i = 0; i < nw; i++)
            if ((out[i] ^ outn) >= GF_P) { ok = 0; break; }
        if (ok) {
            for (uint64_t i = 0; i < nw; i++) out[i] ^= outn;
            *mapping = outn;
            return OR_OK;
        }
        if (ci >= ncands) return OR_MAPPING_FALLBACK;
        outn = cands[ci++];
    }
}

/* internal/rs/gf/map.go:103-113 */
void oracle_map_from_gf(uint32_t n, const uint32_t *in, uint64_t count, uint8_t *out) {
    for (uint64_t i = 0; i < count; i++) {
        uint32_t w = in[i] ^ n;
        out[i * 4] = (uint8_t)(w >> 24);
        out[i * 4 + 1] = (uint8_t)(w >> 16);
        out[i * 4 + 2] = (uint8_t)(w >> 8);
        out[i * 4 + 3] = (uint8_t)w;
    }
}

/* internal/store/multi/multi_store.go:271-299 — returns perVector; parts laid out [count][perVector], zero padded. */
uint64_t oracle_split_vector(const uint32_t *data, uint64_t len, int count, uint32_t *parts) {
    uint64_t per = (len + (uint64_t)count - 1) / (uint64_t)count;
    memset(parts, 0, (size_t)per * count * sizeof(uint32_t));
    if (len) memcpy(parts, data, (size_t)len * sizeof(uint32_t));
    return per;
}

/*
 * The reference's encode framing, multi_store.go:526-531: one CreateParity
 * call per parity row, each re-reading all k data shards (used as the CPU
 * baseline: single-threaded per object, exactly as the reference runs it).
 * shards: object laid out [total][L]; writes rows need..total-1 in place.
 */
int oracle_encode_object(uint32_t *shards, int need, int total, uint64_t L) {
    const uint32_t *data[128];
    uint64_t lens[128];
    if (need > 128) return -1;
    for (int j = 0; j < need; j++) { data[j] = shards + (uint64_t)j * L; lens[j] = L; }
    for (int i = need; i < total; i++) {
        int st = oracle_create_parity(data, lens, need, i, shards + (uint64_t)i * L);
        if (st) return st;
    }
    return OR_OK;
}

/*
 * Per-object timing loop for the CPU baseline's small objects (bench.py):
 * `reps` times the reference's per-object path with its matrix cache
 * (ParityMatrixCached, matrixcache.go:7-29, built once here): r CreateParity
 * calls of one row each (vector.go:18-41) and one RecoverData over the
 * survivors `have` (vector.go:50-88: the inverse built per call, all k rows
 * recomputed).  shards [total][L]; the recovered rows go to scratch [need][L].
 */
int oracle_object_reps(uint32_t *shards, int need, int total, uint64_t L, const int *have, uint32_t *scratch,
                       int reps) {
    const int r = total - need;
    if (need > 128 || total > 256) return -1;
    uint32_t *m = (uint32_t *)malloc((size_t)total * need * sizeof(uint32_t));
    uint32_t *hv = (uint32_t *)malloc((size_t)need * need * sizeof(uint32_t));
    uint32_t *inv = (uint32_t *)malloc((size_t)need * need * sizeof(uint32_t));
    int st = (m && hv && inv) ? oracle_parity_matrix(need, r, m) : -1;
    const uint32_t *data[128], *surv[128];
    uint32_t *out[128];
    for (int j = 0; j < need; j++) {
        data[j] = shards + (uint64_t)j * L;
        surv[j] = shards + (uint64_t)have[j] * L;
        out[j] = scratch + (uint64_t)j * L;
    }
    for (int rep = 0; st == OR_OK && rep < reps; rep++) {
        for (int i = need; i < total; i++) {
            uint32_t *o = shards + (uint64_t)i * L;
            oracle_apply_matrix(m + (size_t)i * need, 1, need, data, &o, L);
        }
        for (int q = 0; q < need; q++) memcpy(hv + (size_t)q * need, m + (size_t)have[q] * need, need * sizeof(uint32_t));
        st = oracle_invert_matrix(hv, need, inv);
        if (st == OR_OK) oracle_apply_matrix(inv, need, need, surv, out, L);
    }
    free(m);
    free(hv);
    free(inv);
    return st;
}

/* Chunk-file header hash of storedir (internal/store/storedir/directory.go:25-28,548-553):
 * fnv.New64a() over SHA-256 ‖ data.  Go's hash/fnv is the published FNV-1a:
 * offset basis 14695981039346656037, prime 1099511628211, h ^= byte then
 * h *= prime (Go standard library, not vendored in the reference; pinned by
 * its published vectors in tests/test_digest.py).  Call with h = the basis
 * to start, and again with the result to continue. */
uint64_t oracle_fnv1a64(uint64_t h, const uint8_t *p, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) {
        h ^= p[i];
        h *= 1099511628211ull;
    }
    return h;
}
