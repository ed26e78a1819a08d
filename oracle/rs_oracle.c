/*
 * CPU oracle + CPU baseline for the CallFS Reed-Solomon path.
 *
 * TEST INFRASTRUCTURE ONLY: linked/loaded solely by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg. The product library (callfs_amd/csrc) never
 * includes or links this file.
 *
 * Restates github.com/klauspost/reedsolomon v1.13.3 (go.mod:13; go.sum:157-158) as
 * called from erasure/codec.go:26-59 — module absent from /root/reference, so this
 * is a from-scratch restatement of the published algorithm:
 *   - GF(2^8) poly 0x11D, generator 2 (upstream galois.go)
 *   - E = V . inv(V[0:k]), V[r][c] = r^c (upstream buildMatrix / matrix.go)
 *   - Encode: parity_j = XOR_i P[j][i]*data_i (codec.go:36)
 *   - Reconstruct with the first-k-present rule (codec.go:55), Verify (codec.go:59)
 * Pinned by the KATs in oracle/rs_oracle.py via tests/test_oracle.py.
 *
 * Two compute paths:
 *   orc_apply_scalar  — log/exp table scalar loop (the checker)
 *   orc_apply_simd    — the CPU baseline ("port"): the upstream SIMD strategy
 *                       (GFNI vgf2p8affineqb 8x8 bit-matrix per coefficient, or AVX2
 *                       split-nibble vpshufb tables, outputs held in registers while
 *                       inputs stream), split by byte range like upstream
 *                       codeSomeShardsP, the ranges run on a persistent thread pool
 *                       (as goroutines reuse runtime threads).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <immintrin.h>

static uint8_t g_exp[512];
static uint8_t g_log[256];
static uint8_t g_mul[256][256];
static int g_init = 0;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void init_tables(void) {
  unsigned x = 1;
  for (int i = 0; i < 255; i++) {
    g_exp[i] = (uint8_t)x;
    g_log[x] = (uint8_t)i;
    x <<= 1;
    if (x & 0x100) x ^= 0x11D;
  }
  for (int i = 255; i < 512; i++) g_exp[i] = g_exp[i - 255];
  for (int a = 0; a < 256; a++)
    for (int b = 0; b < 256; b++)
      g_mul[a][b] = (a == 0 || b == 0) ? 0 : g_exp[g_log[a] + g_log[b]];
  g_init = 1;
}
static void ensure_init(void) { pthread_once(&g_once, init_tables); }

uint8_t orc_gal_mul(uint8_t a, uint8_t b) { ensure_init(); return g_mul[a][b]; }

uint8_t orc_gal_exp(uint8_t a, int n) {
  ensure_init();
  if (n == 0) return 1;
  if (a == 0) return 0;
  return g_exp[(g_log[a] * n) % 255];
}

static uint8_t gal_inv(uint8_t a) { return g_exp[(255 - g_log[a]) % 255]; }

/* Gauss-Jordan over GF(2^8). Returns 0 or -1 when singular. */
int orc_invert(int n, const uint8_t* in, uint8_t* out) {
  ensure_init();
  uint8_t* w = (uint8_t*)malloc((size_t)n * 2 * n);
  for (int r = 0; r < n; r++) {
    memcpy(w + (size_t)r * 2 * n, in + (size_t)r * n, n);
    memset(w + (size_t)r * 2 * n + n, 0, n);
    w[(size_t)r * 2 * n + n + r] = 1;
  }
  for (int r = 0; r < n; r++) {
    uint8_t* row = w + (size_t)r * 2 * n;
    if (row[r] == 0) {
      for (int b = r + 1; b < n; b++) {
        uint8_t* br = w + (size_t)b * 2 * n;
        if (br[r]) {
          for (int c = 0; c < 2 * n; c++) { uint8_t t = row[c]; row[c] = br[c]; br[c] = t; }
          break;
        }
      }
    }
    if (row[r] == 0) { free(w); return -1; }
    uint8_t s = gal_inv(row[r]);
    for (int c = 0; c < 2 * n; c++) row[c] = g_mul[s][row[c]];
    for (int o = 0; o < n; o++) {
      if (o == r) continue;
      uint8_t* orow = w + (size_t)o * 2 * n;
      uint8_t f = orow[r];
      if (!f) continue;
      for (int c = 0; c < 2 * n; c++) orow[c] ^= g_mul[f][row[c]];
    }
  }
  for (int r = 0; r < n; r++) memcpy(out + (size_t)r * n, w + (size_t)r * 2 * n + n, n);
  free(w);
  return 0;
}

/* E = V . inv(V[0:k]); E is (k+m) x k row-major. */
int orc_encode_matrix(int k, int m, uint8_t* E) {
  ensure_init();
  int n = k + m;
  uint8_t* V = (uint8_t*)malloc((size_t)n * k);
  uint8_t* ti = (uint8_t*)malloc((size_t)k * k);
  for (int r = 0; r < n; r++)
    for (int c = 0; c < k; c++) V[(size_t)r * k + c] = orc_gal_exp((uint8_t)r, c);
  if (orc_invert(k, V, ti) != 0) { free(V); free(ti); return -1; }
  for (int r = 0; r < n; r++)
    for (int c = 0; c < k; c++) {
      uint8_t v = 0;
      for (int i = 0; i < k; i++) v ^= g_mul[V[(size_t)r * k + i]][ti[(size_t)i * k + c]];
      E[(size_t)r * k + c] = v;
    }
  free(V); free(ti);
  return 0;
}

/* out_r[b] = XOR_i coef[r*k+i] * in_i[b], scalar (checker). */
void orc_apply_scalar(int rows, int k, const uint8_t* coef, size_t S,
                      const uint8_t* const* in, uint8_t* const* out) {
  ensure_init();
  for (int r = 0; r < rows; r++) {
    uint8_t* o = out[r];
    memset(o, 0, S);
    for (int i = 0; i < k; i++) {
      uint8_t c = coef[(size_t)r * k + i];
      if (!c) continue;
      const uint8_t* mt = g_mul[c];
      const uint8_t* x = in[i];
      for (size_t b = 0; b < S; b++) o[b] ^= mt[x[b]];
    }
  }
}

int orc_encode(int k, int m, size_t S, const uint8_t* const* data, uint8_t* const* parity) {
  if (k < 1 || m < 1 || k + m > 256) return -1;
  uint8_t* E = (uint8_t*)malloc((size_t)(k + m) * k);
  if (orc_encode_matrix(k, m, E)) { free(E); return -1; }
  orc_apply_scalar(m, k, E + (size_t)k * k, S, data, parity);
  free(E);
  return 0;
}

/* Reconstruct missing shards in place (buffers must exist for all n).
 * present[i] != 0 marks present shards. Returns 0, or -2 when fewer than k present. */
int orc_reconstruct(int k, int m, size_t S, uint8_t* const* shards, const uint8_t* present) {
  int n = k + m, np = 0, valid[256];
  for (int i = 0; i < n; i++) if (present[i]) { if (np < k) valid[np] = i; np++; }
  if (np == n) return 0;
  if (np < k) return -2;
  uint8_t* E = (uint8_t*)malloc((size_t)n * k);
  uint8_t* sub = (uint8_t*)malloc((size_t)k * k);
  uint8_t* dec = (uint8_t*)malloc((size_t)k * k);
  orc_encode_matrix(k, m, E);
  for (int r = 0; r < k; r++) memcpy(sub + (size_t)r * k, E + (size_t)valid[r] * k, k);
  if (orc_invert(k, sub, dec)) { free(E); free(sub); free(dec); return -3; }
  const uint8_t* vin[256];
  for (int r = 0; r < k; r++) vin[r] = shards[valid[r]];
  for (int i = 0; i < k; i++)
    if (!present[i]) orc_apply_scalar(1, k, dec + (size_t)i * k, S, vin, &shards[i]);
  const uint8_t* din[256];
  for (int i = 0; i < k; i++) din[i] = shards[i];
  for (int j = 0; j < m; j++)
    if (!present[k + j]) orc_apply_scalar(1, k, E + (size_t)(k + j) * k, S, din, &shards[k + j]);
  free(E); free(sub); free(dec);
  return 0;
}

/* Verify: 1 when parity matches, 0 otherwise. */
int orc_verify(int k, int m, size_t S, const uint8_t* const* shards) {
  uint8_t* E = (uint8_t*)malloc((size_t)(k + m) * k);
  orc_encode_matrix(k, m, E);
  uint8_t* tmp = (uint8_t*)malloc(S ? S : 1);
  int ok = 1;
  for (int j = 0; j < m && ok; j++) {
    uint8_t* o[1] = {tmp};
    orc_apply_scalar(1, k, E + (size_t)(k + j) * k, S, shards, o);
    if (memcmp(tmp, shards[k + j], S) != 0) ok = 0;
  }
  free(tmp); free(E);
  return ok;
}

/* ------------------------------------------------------------------------------------
 * CPU baseline: upstream SIMD strategy, multithreaded by byte range.
 * ------------------------------------------------------------------------------------ */

#define MAX_ROWS_SIMD 8

/* Body with `rows` a compile-time constant at each call site below (always_inline), so
 * the accumulators live in zmm registers like upstream's generated mulGFNI_{k}x{m}. */
__attribute__((target("avx512f,avx512bw,gfni"), always_inline))
static inline void apply_gfni_rows(const int rows, int k, const uint64_t* mats, size_t b0,
                                   size_t b1, const uint8_t* const* in, uint8_t* const* out) {
  size_t b = b0;
  for (; b + 64 <= b1; b += 64) {
    __m512i acc[MAX_ROWS_SIMD];
    for (int r = 0; r < rows; r++) acc[r] = _mm512_setzero_si512();
    for (int i = 0; i < k; i++) {
      __m512i x = _mm512_loadu_si512((const void*)(in[i] + b));
      for (int r = 0; r < rows; r++) {
        __m512i A = _mm512_set1_epi64((long long)mats[(size_t)r * k + i]);
        acc[r] = _mm512_xor_si512(acc[r], _mm512_gf2p8affine_epi64_epi8(x, A, 0));
      }
    }
    for (int r = 0; r < rows; r++) _mm512_storeu_si512((void*)(out[r] + b), acc[r]);
  }
}

__attribute__((target("avx512f,avx512bw,gfni")))
static void apply_gfni_range(int rows, int k, const uint64_t* mats, size_t b0, size_t b1,
                             const uint8_t* const* in, uint8_t* const* out) {
  /* mats[r*k+i] = 8x8 GF(2) bit matrix multiplying by coef[r][i] in GF(2^8)/0x11D */
  switch (rows) {
    case 1: apply_gfni_rows(1, k, mats, b0, b1, in, out); return;
    case 2: apply_gfni_rows(2, k, mats, b0, b1, in, out); return;
    case 3: apply_gfni_rows(3, k, mats, b0, b1, in, out); return;
    case 4: apply_gfni_rows(4, k, mats, b0, b1, in, out); return;
    case 5: apply_gfni_rows(5, k, mats, b0, b1, in, out); return;
    case 6: apply_gfni_rows(6, k, mats, b0, b1, in, out); return;
    case 7: apply_gfni_rows(7, k, mats, b0, b1, in, out); return;
    default: break;
  }
  size_t b = b0;
  for (; b + 64 <= b1; b += 64) {
    __m512i acc[MAX_ROWS_SIMD];
    for (int r = 0; r < rows; r++) acc[r] = _mm512_setzero_si512();
    for (int i = 0; i < k; i++) {
      __m512i x = _mm512_loadu_si512((const void*)(in[i] + b));
      for (int r = 0; r < rows; r++) {
        __m512i A = _mm512_set1_epi64((long long)mats[(size_t)r * k + i]);
        acc[r] = _mm512_xor_si512(acc[r], _mm512_gf2p8affine_epi64_epi8(x, A, 0));
      }
    }
    for (int r = 0; r < rows; r++) _mm512_storeu_si512((void*)(out[r] + b), acc[r]);
  }
  (void)b;
}

__attribute__((target("avx2")))
static void apply_avx2_range(int rows, int k, const uint8_t* lo_tab, const uint8_t* hi_tab,
                             size_t b0, size_t b1, const uint8_t* const* in, uint8_t* const* out) {
  /* lo_tab/hi_tab: (r*k+i)*16 nibble tables, as upstream mulAvxTwo */
  const __m256i mask = _mm256_set1_epi8(0x0f);
  size_t b = b0;
  for (; b + 32 <= b1; b += 32) {
    __m256i acc[MAX_ROWS_SIMD];
    for (int r = 0; r < rows; r++) acc[r] = _mm256_setzero_si256();
    for (int i = 0; i < k; i++) {
      __m256i x = _mm256_loadu_si256((const __m256i*)(in[i] + b));
      __m256i lo = _mm256_and_si256(x, mask);
      __m256i hi = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
      for (int r = 0; r < rows; r++) {
        const uint8_t* lt = lo_tab + ((size_t)r * k + i) * 16;
        const uint8_t* ht = hi_tab + ((size_t)r * k + i) * 16;
        __m256i L = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)lt));
        __m256i H = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)ht));
        acc[r] = _mm256_xor_si256(acc[r], _mm256_xor_si256(_mm256_shuffle_epi8(L, lo),
                                                           _mm256_shuffle_epi8(H, hi)));
      }
    }
    for (int r = 0; r < rows; r++) _mm256_storeu_si256((__m256i*)(out[r] + b), acc[r]);
  }
}

static uint64_t gfni_matrix(uint8_t c) {
  /* byte (7-i) holds the row producing output bit i: bit b set iff bit i of c*2^b */
  uint64_t A = 0;
  for (int i = 0; i < 8; i++) {
    uint8_t row = 0;
    for (int b = 0; b < 8; b++)
      if ((g_mul[c][1u << b] >> i) & 1) row |= (uint8_t)(1u << b);
    A |= (uint64_t)row << (8 * (7 - i));
  }
  return A;
}

int orc_simd_kind(void) {
  __builtin_cpu_init();
  if (__builtin_cpu_supports("gfni") && __builtin_cpu_supports("avx512bw")) return 2;
  if (__builtin_cpu_supports("avx2")) return 1;
  return 0;
}

typedef struct {
  int rows, k, kind;
  const uint8_t* coef;
  const uint64_t* mats;
  const uint8_t* lo;
  const uint8_t* hi;
  size_t b0, b1;
  const uint8_t* const* in;
  uint8_t* const* out;
} job_t;

static void run_range(const job_t* j) {
  size_t b = j->b0;
  size_t vec = j->kind == 2 ? 64 : (j->kind == 1 ? 32 : 1);
  size_t bulk = j->b0 + (j->b1 - j->b0) / vec * vec;
  if (j->kind == 2) apply_gfni_range(j->rows, j->k, j->mats, j->b0, bulk, j->in, j->out);
  else if (j->kind == 1) apply_avx2_range(j->rows, j->k, j->lo, j->hi, j->b0, bulk, j->in, j->out);
  else bulk = j->b0;
  for (b = bulk; b < j->b1; b++) {
    for (int r = 0; r < j->rows; r++) {
      uint8_t v = 0;
      for (int i = 0; i < j->k; i++) v ^= g_mul[j->coef[(size_t)r * j->k + i]][j->in[i][b]];
      j->out[r][b] = v;
    }
  }
}

/* Persistent worker pool (the Go runtime reuses goroutine threads; spawning pthreads
 * per call cost ~10-20 us each). Workers take job indices from an atomic counter; the
 * caller takes jobs too and returns when every job is done. One call at a time. */
#define POOL_MAX 256
static struct {
  pthread_mutex_t mu;
  pthread_cond_t go, done;
  int nworkers, gen, pending;
  job_t* jobs;
  int njobs;
  int next;  /* guarded by mu */
} g_pool = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, PTHREAD_COND_INITIALIZER,
            0, 0, 0, NULL, 0, 0};
static pthread_mutex_t g_call = PTHREAD_MUTEX_INITIALIZER;

static int pool_take(void) {
  pthread_mutex_lock(&g_pool.mu);
  int t = g_pool.next < g_pool.njobs ? g_pool.next++ : -1;
  pthread_mutex_unlock(&g_pool.mu);
  return t;
}

static void pool_finish(void) {
  pthread_mutex_lock(&g_pool.mu);
  if (--g_pool.pending == 0) pthread_cond_broadcast(&g_pool.done);
  pthread_mutex_unlock(&g_pool.mu);
}

static void* pool_worker(void* arg) {
  (void)arg;
  int seen = 0;
  for (;;) {
    pthread_mutex_lock(&g_pool.mu);
    while (g_pool.gen == seen) pthread_cond_wait(&g_pool.go, &g_pool.mu);
    seen = g_pool.gen;
    pthread_mutex_unlock(&g_pool.mu);
    for (int t; (t = pool_take()) >= 0;) {
      run_range(&g_pool.jobs[t]);
      pool_finish();
    }
  }
  return NULL;
}

static void pool_run(job_t* jobs, int njobs) {
  pthread_mutex_lock(&g_call);
  pthread_mutex_lock(&g_pool.mu);
  while (g_pool.nworkers < njobs - 1 && g_pool.nworkers < POOL_MAX) {
    pthread_t th;
    if (pthread_create(&th, NULL, pool_worker, NULL) != 0) break;
    pthread_detach(th);
    g_pool.nworkers++;
  }
  g_pool.jobs = jobs;
  g_pool.njobs = njobs;
  g_pool.next = 0;
  g_pool.pending = njobs;
  g_pool.gen++;
  pthread_cond_broadcast(&g_pool.go);
  pthread_mutex_unlock(&g_pool.mu);
  for (int t; (t = pool_take()) >= 0;) {
    run_range(&jobs[t]);
    pool_finish();
  }
  pthread_mutex_lock(&g_pool.mu);
  while (g_pool.pending > 0) pthread_cond_wait(&g_pool.done, &g_pool.mu);
  g_pool.jobs = NULL;
  g_pool.njobs = 0;
  pthread_mutex_unlock(&g_pool.mu);
  pthread_mutex_unlock(&g_call);
}

/* CPU baseline entry point. Rows are processed MAX_ROWS_SIMD at a time. */
void orc_apply_simd(int rows, int k, const uint8_t* coef, size_t S,
                    const uint8_t* const* in, uint8_t* const* out, int nthreads) {
  ensure_init();
  int kind = orc_simd_kind();
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  for (int r0 = 0; r0 < rows; r0 += MAX_ROWS_SIMD) {
    int rr = rows - r0 < MAX_ROWS_SIMD ? rows - r0 : MAX_ROWS_SIMD;
    const uint8_t* cf = coef + (size_t)r0 * k;
    size_t nt = (size_t)rr * k;
    uint64_t* mats = (uint64_t*)malloc(nt * sizeof(uint64_t));
    uint8_t* lo = (uint8_t*)malloc(nt * 16);
    uint8_t* hi = (uint8_t*)malloc(nt * 16);
    for (size_t t = 0; t < nt; t++) {
      mats[t] = gfni_matrix(cf[t]);
      for (int x = 0; x < 16; x++) {
        lo[t * 16 + x] = g_mul[cf[t]][x];
        hi[t * 16 + x] = g_mul[cf[t]][x << 4];
      }
    }
    /* byte ranges: 64-B aligned, like upstream codeSomeShardsP */
    size_t per = (S + nthreads - 1) / nthreads;
    per = (per + 63) & ~(size_t)63;
    if (per < 4096) per = 4096;
    int njobs = (int)((S + per - 1) / per);
    if (njobs < 1) njobs = 1;
    job_t* jobs = (job_t*)calloc((size_t)njobs, sizeof(job_t));
    for (int t = 0; t < njobs; t++) {
      jobs[t].rows = rr; jobs[t].k = k; jobs[t].kind = kind;
      jobs[t].coef = cf; jobs[t].mats = mats; jobs[t].lo = lo; jobs[t].hi = hi;
      jobs[t].b0 = (size_t)t * per;
      jobs[t].b1 = (size_t)(t + 1) * per < S ? (size_t)(t + 1) * per : S;
      jobs[t].in = in; jobs[t].out = out + r0;
    }
    if (njobs == 1) run_range(&jobs[0]);
    else pool_run(jobs, njobs);
    free(jobs); free(mats); free(lo); free(hi);
  }
}

/* ------------------------------------------------------------------------------------
 * CPU baseline driver: the reference's per-object work timed natively (no per-shard
 * Python calls). For each stripe of a [stripe][n][S] buffer:
 *   ops & 1  Encode       parity = P . data                        (codec.go:36)
 *   ops & 2  Reconstruct  erased data from the first k present,
 *                         then erased parity from data             (codec.go:55)
 *   ops & 4  Verify       P . data into a temporary, compared with
 *                         the stored parity (bytes.Equal)          (codec.go:59)
 * Erased shards are rewritten in place (upstream reuses a nil entry's capacity).
 * mode 0 "stripe-parallel": each thread takes whole stripes (independent requests on
 *        separate goroutines, manager.go:60 shares one Codec);
 * mode 1 "byte-range": every op of every stripe is split over all threads by 64-B
 *        aligned byte ranges with a join after each op (upstream codeSomeShardsP).
 * Returns the number of Verify mismatches (stripes x parity rows), or < 0 on error.
 * ------------------------------------------------------------------------------------ */

typedef struct {
  int rows, k;
  uint8_t coef[MAX_ROWS_SIMD * 256];
  uint64_t mats[MAX_ROWS_SIMD * 256];
  uint8_t lo[MAX_ROWS_SIMD * 256 * 16], hi[MAX_ROWS_SIMD * 256 * 16];
} rowset_t;

static void rowset_prep(rowset_t* rs, int rows, int k, const uint8_t* coef) {
  rs->rows = rows;
  rs->k = k;
  for (int t = 0; t < rows * k; t++) {
    rs->coef[t] = coef[t];
    rs->mats[t] = gfni_matrix(coef[t]);
    for (int x = 0; x < 16; x++) {
      rs->lo[t * 16 + x] = g_mul[coef[t]][x];
      rs->hi[t * 16 + x] = g_mul[coef[t]][x << 4];
    }
  }
}

static void rowset_apply(const rowset_t* rs, int kind, size_t b0, size_t b1,
                         const uint8_t* const* in, uint8_t* const* out) {
  job_t j;
  j.rows = rs->rows; j.k = rs->k; j.kind = kind;
  j.coef = rs->coef; j.mats = rs->mats; j.lo = rs->lo; j.hi = rs->hi;
  j.b0 = b0; j.b1 = b1; j.in = in; j.out = out;
  run_range(&j);
}

#define BENCH_MAX_SETS 64 /* ceil(256 / MAX_ROWS_SIMD) row sets per matrix */

typedef struct {
  int k, m, n, kind, ops, mode, nthreads;
  size_t S, stripe_pitch, shard_pitch;
  uint8_t* buf;
  int nstripes;
  int valid[256], nmiss_d, miss_d[256], nmiss_p, miss_p[256];
  rowset_t* enc;  int nenc;   /* P, MAX_ROWS_SIMD rows per set */
  rowset_t* dec;  int ndec;   /* inv(E[valid]) rows of the erased data shards */
  rowset_t* par;  int npar;   /* P rows of the erased parity shards */
  uint8_t** tmp;              /* per-thread m x S verify temporaries (mode 0) or one */
  /* phase state */
  pthread_barrier_t start, end;
  volatile int stop;
  int cur_stripe, cur_op, njobs;
  size_t per;
  int next; /* atomic */
  int mismatches; /* atomic */
  pthread_mutex_t* gate;
} bench_t;

static void bench_op(bench_t* B, int s, int op, size_t b0, size_t b1, uint8_t* tmp) {
  uint8_t* base = B->buf + (size_t)s * B->stripe_pitch;
  const uint8_t* in[256];
  uint8_t* out[256];
  for (int i = 0; i < B->n; i++) in[i] = base + (size_t)i * B->shard_pitch;
  if (op == 1) {
    for (int g = 0; g < B->nenc; g++) {
      for (int r = 0; r < B->enc[g].rows; r++)
        out[r] = base + (size_t)(B->k + g * MAX_ROWS_SIMD + r) * B->shard_pitch;
      rowset_apply(&B->enc[g], B->kind, b0, b1, in, out);
    }
  } else if (op == 2) {
    const uint8_t* vin[256];
    for (int i = 0; i < B->k; i++) vin[i] = in[B->valid[i]];
    for (int g = 0; g < B->ndec; g++) {
      for (int r = 0; r < B->dec[g].rows; r++)
        out[r] = base + (size_t)B->miss_d[g * MAX_ROWS_SIMD + r] * B->shard_pitch;
      rowset_apply(&B->dec[g], B->kind, b0, b1, vin, out);
    }
    for (int g = 0; g < B->npar; g++) {
      for (int r = 0; r < B->par[g].rows; r++)
        out[r] = base + (size_t)B->miss_p[g * MAX_ROWS_SIMD + r] * B->shard_pitch;
      rowset_apply(&B->par[g], B->kind, b0, b1, in, out);
    }
  } else if (op == 4) {
    for (int g = 0; g < B->nenc; g++) {
      for (int r = 0; r < B->enc[g].rows; r++)
        out[r] = tmp + (size_t)(g * MAX_ROWS_SIMD + r) * B->S;
      rowset_apply(&B->enc[g], B->kind, b0, b1, in, out);
    }
    int bad = 0;
    for (int j = 0; j < B->m; j++)
      bad += memcmp(tmp + (size_t)j * B->S + b0, in[B->k + j] + b0, b1 - b0) != 0;
    if (bad) __atomic_fetch_add(&B->mismatches, bad, __ATOMIC_RELAXED);
  }
}

static void bench_work(bench_t* B, int tid) {
  for (;;) {
    int j = __atomic_fetch_add(&B->next, 1, __ATOMIC_RELAXED);
    if (j >= B->njobs) return;
    if (B->mode == 0) {
      for (int op = 1; op <= 4; op <<= 1)
        if (B->ops & op) bench_op(B, j, op, 0, B->S, B->tmp[tid]);
    } else {
      size_t b0 = (size_t)j * B->per, b1 = b0 + B->per < B->S ? b0 + B->per : B->S;
      bench_op(B, B->cur_stripe, B->cur_op, b0, b1, B->tmp[0]);
    }
  }
}

typedef struct { bench_t* B; int tid; } bench_arg_t;

static void* bench_thread(void* p) {
  bench_arg_t* a = (bench_arg_t*)p;
  pthread_mutex_lock(a->B->gate); /* wait until the barriers are initialised */
  pthread_mutex_unlock(a->B->gate);
  for (;;) {
    pthread_barrier_wait(&a->B->start);
    if (a->B->stop) return NULL;
    bench_work(a->B, a->tid);
    pthread_barrier_wait(&a->B->end);
  }
}

/* One phase on all threads: `njobs` jobs (stripes in mode 0, byte ranges in mode 1). */
static void bench_phase(bench_t* B, int njobs) {
  B->njobs = njobs;
  __atomic_store_n(&B->next, 0, __ATOMIC_RELAXED);
  pthread_barrier_wait(&B->start);
  bench_work(B, 0);
  pthread_barrier_wait(&B->end);
}

static void bench_pass(bench_t* B) {
  if (B->mode == 0) {
    bench_phase(B, B->nstripes);
    return;
  }
  const int nr = (int)((B->S + B->per - 1) / B->per);
  for (int s = 0; s < B->nstripes; s++)
    for (int op = 1; op <= 4; op <<= 1)
      if (B->ops & op) {
        B->cur_stripe = s;
        B->cur_op = op;
        bench_phase(B, nr);
      }
}

static double mono_now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + (double)t.tv_nsec * 1e-9;
}

static rowset_t* make_sets(int rows, int k, const uint8_t* coef, int* nsets) {
  *nsets = (rows + MAX_ROWS_SIMD - 1) / MAX_ROWS_SIMD;
  if (*nsets == 0) return NULL;
  rowset_t* s = (rowset_t*)calloc((size_t)*nsets, sizeof(rowset_t));
  for (int g = 0; g < *nsets; g++) {
    int rr = rows - g * MAX_ROWS_SIMD < MAX_ROWS_SIMD ? rows - g * MAX_ROWS_SIMD : MAX_ROWS_SIMD;
    rowset_prep(&s[g], rr, k, coef + (size_t)g * MAX_ROWS_SIMD * k);
  }
  return s;
}

int orc_bench_codec(int k, int m, size_t S, uint8_t* buf, size_t stripe_pitch,
                    size_t shard_pitch, int nstripes, const uint8_t* present, int ops,
                    int mode, int nthreads, double seconds, double* elapsed_out,
                    int* passes_out) {
  ensure_init();
  if (k < 1 || m < 1 || k + m > 256 || !buf || nstripes < 1 || S == 0 || nthreads < 1 ||
      nthreads > POOL_MAX || (mode != 0 && mode != 1))
    return -1;
  bench_t* B = (bench_t*)calloc(1, sizeof(bench_t));
  B->k = k; B->m = m; B->n = k + m; B->S = S; B->buf = buf;
  B->stripe_pitch = stripe_pitch; B->shard_pitch = shard_pitch; B->nstripes = nstripes;
  B->ops = ops; B->mode = mode; B->nthreads = nthreads; B->kind = orc_simd_kind();
  uint8_t* E = (uint8_t*)malloc((size_t)B->n * k);
  uint8_t* sub = (uint8_t*)malloc((size_t)k * k);
  uint8_t* inv = (uint8_t*)malloc((size_t)k * k);
  uint8_t* drows = (uint8_t*)malloc((size_t)k * k);
  uint8_t* prows = (uint8_t*)malloc((size_t)m * k);
  int rc = -1;
  if (orc_encode_matrix(k, m, E)) goto out;
  int np = 0;
  for (int i = 0; i < B->n; i++)
    if (!present || present[i]) { if (np < k) B->valid[np] = i; np++; }
  if (np < k) { rc = -2; goto out; }
  for (int r = 0; r < k; r++) memcpy(sub + (size_t)r * k, E + (size_t)B->valid[r] * k, k);
  if (orc_invert(k, sub, inv)) { rc = -3; goto out; }
  for (int i = 0; i < B->n; i++) {
    if (present && present[i]) continue;
    if (!present) break;
    if (i < k) {
      memcpy(drows + (size_t)B->nmiss_d * k, inv + (size_t)i * k, k);
      B->miss_d[B->nmiss_d++] = i;
    } else {
      memcpy(prows + (size_t)B->nmiss_p * k, E + (size_t)i * k, k);
      B->miss_p[B->nmiss_p++] = i;
    }
  }
  B->enc = make_sets(m, k, E + (size_t)k * k, &B->nenc);
  B->dec = make_sets(B->nmiss_d, k, drows, &B->ndec);
  B->par = make_sets(B->nmiss_p, k, prows, &B->npar);
  const int ntmp = nthreads;
  B->tmp = (uint8_t**)calloc((size_t)nthreads, sizeof(uint8_t*));
  for (int t = 0; t < (mode == 0 ? nthreads : 1); t++) B->tmp[t] = (uint8_t*)malloc((size_t)m * S);
  /* byte ranges: 64-B aligned, at least 4 KiB, one per thread */
  B->per = (S + nthreads - 1) / nthreads;
  B->per = (B->per + 63) & ~(size_t)63;
  if (B->per < 4096) B->per = 4096;
  /* the barriers count the threads that exist: if the system refuses a thread, run
   * with the ones created so far instead of waiting forever at the first barrier */
  pthread_t th[POOL_MAX];
  bench_arg_t args[POOL_MAX];
  pthread_mutex_t gate = PTHREAD_MUTEX_INITIALIZER;
  pthread_mutex_lock(&gate); /* held until the barriers exist */
  int made = 1;
  B->gate = &gate;
  for (int t = 1; t < nthreads; t++) {
    args[t].B = B;
    args[t].tid = t;
    if (pthread_create(&th[t], NULL, bench_thread, &args[t]) != 0) break;
    made++;
  }
  nthreads = made;
  B->nthreads = made;
  pthread_barrier_init(&B->start, NULL, (unsigned)nthreads);
  pthread_barrier_init(&B->end, NULL, (unsigned)nthreads);
  pthread_mutex_unlock(&gate);
  int passes = 0;
  const double t0 = mono_now();
  double el;
  do {
    bench_pass(B);
    passes++;
  } while ((el = mono_now() - t0) < seconds);
  B->stop = 1;
  pthread_barrier_wait(&B->start);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
  pthread_barrier_destroy(&B->start);
  pthread_barrier_destroy(&B->end);
  if (elapsed_out) *elapsed_out = el;
  if (passes_out) *passes_out = passes;
  rc = B->mismatches;
  for (int t = 0; t < ntmp; t++) free(B->tmp[t]);
  free(B->tmp);
  free(B->enc); free(B->dec); free(B->par);
out:
  free(E); free(sub); free(inv); free(drows); free(prows);
  free(B);
  return rc;
}
