/* Drives rs_codec_encode / rs_codec_decode exactly as the cgo shim does
 * (go/erasure/codec_rocm.go): a C-malloc'd pointer array over separately allocated
 * shard buffers, a C-malloc'd lens array with 0 for nil entries, and every error path
 * of codec.go:45-78 in its precedence order.
 *
 * The contract checked on every error path before Reconstruct has run (shard count,
 * size mismatch, no data, too few shards): no lens[i] changes and no missing-shard
 * buffer is written, so the shim can leave the caller's [][]byte untouched, as
 * upstream Reconstruct does.
 *
 * Without a HIP device (rs_init -> RS_E_HIP) only those argument paths run, against a
 * context pointer the library must not dereference on them (tests/test_native_cgo.py
 * builds this with -fsanitize=address,undefined on the CPU). With a device the same
 * binary also runs the round trips, each checked against the C oracle
 * (oracle/rs_oracle.c, linked as the checker only).
 *
 * usage: cgo_drive [gpu]   ("gpu": fail unless a device is present) */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "callfs_rs.h"

int orc_encode(int k, int m, size_t S, const uint8_t* const* data, uint8_t* const* parity);

static int fails = 0;
#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);      \
      ++fails;                                                \
    }                                                         \
  } while (0)

#define SENTINEL 0xA5

/* The shim's view of one Decode call: n C-allocated entries, missing ones with a
 * buffer of S bytes filled with SENTINEL and lens 0. */
typedef struct {
  int n;
  uint8_t** ptrs;
  size_t* lens;
  size_t* lens0;
  size_t S;
} call_t;

static call_t make_call(int n, size_t S, uint8_t* const* shards, const int* missing_mask,
                        const size_t* len_override) {
  call_t c;
  c.n = n;
  c.S = S;
  c.ptrs = (uint8_t**)malloc(sizeof(uint8_t*) * (size_t)n);
  c.lens = (size_t*)malloc(sizeof(size_t) * (size_t)n);
  c.lens0 = (size_t*)malloc(sizeof(size_t) * (size_t)n);
  for (int i = 0; i < n; i++) {
    size_t L = len_override ? len_override[i] : S;
    c.ptrs[i] = (uint8_t*)malloc(S ? S : 1);
    if (missing_mask[i] || L == 0) {
      memset(c.ptrs[i], SENTINEL, S);
      c.lens[i] = 0;
    } else {
      memcpy(c.ptrs[i], shards[i], L < S ? L : S);
      c.lens[i] = L;
    }
    c.lens0[i] = c.lens[i];
  }
  return c;
}

static int untouched(const call_t* c) {
  for (int i = 0; i < c->n; i++) {
    if (c->lens[i] != c->lens0[i]) return 0;
    if (c->lens0[i] == 0)
      for (size_t b = 0; b < c->S; b++)
        if (c->ptrs[i][b] != SENTINEL) return 0;
  }
  return 1;
}

static void free_call(call_t* c) {
  for (int i = 0; i < c->n; i++) free(c->ptrs[i]);
  free(c->ptrs);
  free(c->lens);
  free(c->lens0);
}

/* Error paths that return before any device work. */
static void argument_paths(rs_ctx* ctx, int k, int m, size_t S, uint8_t* const* shards) {
  const int n = k + m;
  int* miss = (int*)calloc((size_t)n, sizeof(int));
  uint8_t out[64];

  /* profile first (codec.go:46-48), whatever the shards look like */
  {
    for (int i = 0; i < n; i++) miss[i] = i < m + 1;
    call_t c = make_call(n, S, shards, miss, NULL);
    CHECK(rs_codec_decode(ctx, 0, m, c.ptrs, c.lens, out, 16) == RS_E_INVALID_PROFILE);
    CHECK(rs_codec_decode(ctx, k, 0, c.ptrs, c.lens, out, 16) == RS_E_INVALID_PROFILE);
    CHECK(untouched(&c));
    free_call(&c);
  }
  /* too few shards: m+1 missing (codec_test.go:65-88) */
  {
    for (int i = 0; i < n; i++) miss[i] = i >= n - (m + 1);
    call_t c = make_call(n, S, shards, miss, NULL);
    CHECK(rs_codec_decode(ctx, k, m, c.ptrs, c.lens, out, 16) == RS_E_TOO_FEW_SHARDS);
    CHECK(untouched(&c));
    CHECK(rs_reconstruct(ctx, k, m, c.ptrs, c.lens) == RS_E_TOO_FEW_SHARDS);
    CHECK(untouched(&c));
    free_call(&c);
  }
  /* every entry nil: upstream ErrShardNoData */
  {
    for (int i = 0; i < n; i++) miss[i] = 1;
    call_t c = make_call(n, S, shards, miss, NULL);
    CHECK(rs_codec_decode(ctx, k, m, c.ptrs, c.lens, out, 16) == RS_E_NO_DATA);
    CHECK(untouched(&c));
    free_call(&c);
  }
  /* one short shard beside a missing one: ErrShardSize before the count check */
  if (S >= 2) {
    size_t* ln = (size_t*)malloc(sizeof(size_t) * (size_t)n);
    for (int i = 0; i < n; i++) {
      miss[i] = i == 0;
      ln[i] = i == n - 1 ? S - 1 : S;
    }
    call_t c = make_call(n, S, shards, miss, ln);
    CHECK(rs_codec_decode(ctx, k, m, c.ptrs, c.lens, out, 16) == RS_E_SHARD_SIZE);
    CHECK(untouched(&c));
    free_call(&c);
    /* size mismatch wins over too few as well */
    for (int i = 0; i < n; i++) miss[i] = i < m + 1;
    c = make_call(n, S, shards, miss, ln);
    CHECK(rs_codec_decode(ctx, k, m, c.ptrs, c.lens, out, 16) == RS_E_SHARD_SIZE);
    CHECK(untouched(&c));
    free_call(&c);
    free(ln);
  }
  /* RepairBatch (rs_reconstruct_batch): per-stripe statuses vs call-level RS_E_ARG. Stripe 0
     lacks m+1 shards, stripe 1 has a present entry with a nil pointer; neither touches the
     device, lens stays as it was, and a call-level error writes no status at all. */
  {
    uint8_t** bp = (uint8_t**)malloc(sizeof(uint8_t*) * 2 * (size_t)n);
    size_t* bl = (size_t*)malloc(sizeof(size_t) * 2 * (size_t)n);
    for (int i = 0; i < n; i++) {
      const int gone = i >= n - (m + 1);
      bp[i] = gone ? NULL : shards[i];
      bl[i] = gone ? 0 : S;
      bp[n + i] = i == n - 1 ? NULL : shards[i];
      bl[n + i] = S;
    }
    int st[2] = {-12345, -12345};
    CHECK(rs_reconstruct_batch(ctx, k, m, 2, bp, bl, 1, st) == RS_E_TOO_FEW_SHARDS);
    CHECK(st[0] == RS_E_TOO_FEW_SHARDS && st[1] == RS_E_ARG);
    for (int i = 0; i < n; i++) CHECK(bl[i] == (i >= n - (m + 1) ? 0 : S) && bl[n + i] == S);
    st[0] = st[1] = -12345;
    CHECK(rs_reconstruct_batch(ctx, k, m, 2, bp, bl, 1, NULL) == RS_E_ARG);
    CHECK(rs_reconstruct_batch(NULL, k, m, 2, bp, bl, 1, st) == RS_E_ARG);
    CHECK(st[0] == -12345 && st[1] == -12345); /* the shim tells call-level from per-stripe so */
    free(bl);
    free(bp);
  }
  /* encode: empty object (Split -> ErrShortData), also for a k+m > 256 profile */
  {
    size_t ss = 7;
    uint8_t buf[8];
    CHECK(rs_codec_encode(ctx, k, m, NULL, 0, NULL, 0, &ss) == RS_E_SHORT_DATA);
    CHECK(rs_codec_encode(ctx, 200, 100, NULL, 0, NULL, 0, &ss) == RS_E_SHORT_DATA);
    CHECK(rs_codec_encode(ctx, 200, 100, buf, 1, buf, 8, &ss) == RS_E_UNSUPPORTED);
    CHECK(rs_codec_encode(ctx, 0, m, buf, 1, buf, 8, &ss) == RS_E_INVALID_PROFILE);
    CHECK(ss == 7); /* not written on error */
  }
  /* pinned host buffers (the shim's HostBuffer / BodyBuffer / FreeHostBuffer): bad
     arguments return before the context is touched */
  {
    void* p = (void*)0x1;
    CHECK(rs_host_alloc(NULL, 16, &p) == RS_E_ARG);
    CHECK(rs_host_alloc(ctx, 0, &p) == RS_E_ARG);
    CHECK(rs_host_alloc(ctx, 16, NULL) == RS_E_ARG);
    CHECK(rs_host_free(NULL, out) == RS_E_ARG);
    CHECK(rs_host_free(ctx, NULL) == RS_E_ARG);
  }
  free(miss);
}

static uint32_t lcg(uint32_t* s) {
  *s = *s * 1664525u + 1013904223u;
  return *s >> 24;
}

/* Encode -> erase -> Decode round trips on the device, against the oracle. */
static void device_paths(rs_ctx* ctx, int k, int m, size_t L) {
  const int n = k + m;
  uint8_t* data = (uint8_t*)malloc(L);
  uint32_t seed = (uint32_t)(L * 31u + (unsigned)k);
  for (size_t i = 0; i < L; i++) data[i] = (uint8_t)lcg(&seed);
  const size_t S = (L + (size_t)k - 1) / (size_t)k;
  uint8_t* all = (uint8_t*)malloc(S * (size_t)n);
  size_t ss = 0;
  CHECK(rs_codec_encode(ctx, k, m, data, L, all, S * (size_t)n, &ss) == RS_OK);
  CHECK(ss == S);
  /* oracle parity from the Split layout */
  uint8_t* padded = (uint8_t*)calloc(S * (size_t)k, 1);
  memcpy(padded, data, L);
  const uint8_t** din = (const uint8_t**)malloc(sizeof(uint8_t*) * (size_t)k);
  uint8_t** pout = (uint8_t**)malloc(sizeof(uint8_t*) * (size_t)m);
  uint8_t* want = (uint8_t*)malloc(S * (size_t)m);
  for (int i = 0; i < k; i++) din[i] = padded + S * (size_t)i;
  for (int j = 0; j < m; j++) pout[j] = want + S * (size_t)j;
  CHECK(orc_encode(k, m, S, din, pout) == 0);
  CHECK(memcmp(all, padded, S * (size_t)k) == 0);
  CHECK(memcmp(all + S * (size_t)k, want, S * (size_t)m) == 0);
  uint8_t** shards = (uint8_t**)malloc(sizeof(uint8_t*) * (size_t)n);
  for (int i = 0; i < n; i++) shards[i] = all + S * (size_t)i;

  argument_paths(ctx, k, m, S, shards);

  int* miss = (int*)calloc((size_t)n, sizeof(int));
  uint8_t* out = (uint8_t*)malloc(L);
  /* m erasures spread over data and parity: reconstructed into the nil entries */
  for (int i = 0; i < n; i++) miss[i] = (i % 3 == 0) && i < 3 * m;
  {
    call_t c = make_call(n, S, shards, miss, NULL);
    memset(out, 0, L);
    CHECK(rs_codec_decode(ctx, k, m, c.ptrs, c.lens, out, (int64_t)L) == RS_OK);
    CHECK(memcmp(out, data, L) == 0);
    for (int i = 0; i < n; i++) {
      CHECK(c.lens[i] == S);
      CHECK(memcmp(c.ptrs[i], shards[i], S) == 0);
    }
    free_call(&c);
  }
  /* a flipped byte in parity that is present beyond the first k: ErrShardCorrupted */
  {
    for (int i = 0; i < n; i++) miss[i] = i == 1;
    call_t c = make_call(n, S, shards, miss, NULL);
    c.ptrs[n - 1][S / 2] ^= 0x40;
    CHECK(rs_codec_decode(ctx, k, m, c.ptrs, c.lens, out, (int64_t)L) == RS_E_CORRUPT);
    CHECK(c.lens[1] == S); /* Reconstruct ran: the entry was filled, as upstream */
    free_call(&c);
  }
  /* originalSize beyond k*S: ErrInsufficientShards after a clean reconstruct+verify */
  {
    for (int i = 0; i < n; i++) miss[i] = 0;
    call_t c = make_call(n, S, shards, miss, NULL);
    uint8_t* big = (uint8_t*)malloc(S * (size_t)k + 1);
    CHECK(rs_codec_decode(ctx, k, m, c.ptrs, c.lens, big, (int64_t)(S * (size_t)k + 1)) ==
          RS_E_INSUFFICIENT);
    free(big);
    free_call(&c);
  }
  free(out); free(miss); free(shards); free(want); free(pout); free(din); free(padded);
  free(all); free(data);
}

/* The shim's pinned-body contract (codec_rocm.go BodyBuffer, Encode, DecodePinned,
 * FreeHostBuffer): allocate a body with room for all n shards, fill it, Split in place
 * (zero padding past L), encode with every shard inside the one allocation (zero-copy);
 * decode from shards fetched into host buffers into host buffers; free everything; the
 * next request of the same size gets the freed body back from the context's pool. */
static void host_body_paths(rs_ctx* ctx, int k, int m, size_t L, int same_body) {
  const int n = k + m;
  const size_t S = (L + (size_t)k - 1) / (size_t)k;
  void* first = NULL;
  for (int round = 0; round < 2; round++) {
    uint8_t* body = NULL;
    CHECK(rs_host_alloc(ctx, S * (size_t)n, (void**)&body) == RS_OK && body != NULL);
    if (!body) return;
    if (round == 0) first = body;
    else if (same_body) CHECK((void*)body == first); /* the freed body came back (the only
                                                         kept buffer of its size class) */
    uint32_t seed = (uint32_t)(L + 17u * (unsigned)round);
    for (size_t i = 0; i < L; i++) body[i] = (uint8_t)lcg(&seed);
    memset(body + L, 0, S * (size_t)n - L); /* Split zeroes the spare capacity */
    const uint8_t** din = (const uint8_t**)malloc(sizeof(uint8_t*) * (size_t)k);
    uint8_t** pout = (uint8_t**)malloc(sizeof(uint8_t*) * (size_t)m);
    uint8_t* want = (uint8_t*)malloc(S * (size_t)m);
    for (int i = 0; i < k; i++) din[i] = body + S * (size_t)i;
    for (int j = 0; j < m; j++) pout[j] = body + S * (size_t)(k + j);
    CHECK(rs_encode(ctx, k, m, S, din, pout) == RS_OK);
    for (int j = 0; j < m; j++) pout[j] = want + S * (size_t)j;
    CHECK(orc_encode(k, m, S, din, pout) == 0);
    CHECK(memcmp(body + S * (size_t)k, want, S * (size_t)m) == 0);
    /* DecodePinned: fetched shards, the reconstructed entries and the object pinned too */
    uint8_t** sh = (uint8_t**)malloc(sizeof(uint8_t*) * (size_t)n);
    size_t* lens = (size_t*)malloc(sizeof(size_t) * (size_t)n);
    for (int i = 0; i < n; i++) {
      CHECK(rs_host_alloc(ctx, S, (void**)&sh[i]) == RS_OK);
      if (i % 4 == 1) {
        memset(sh[i], SENTINEL, S);
        lens[i] = 0;
      } else {
        memcpy(sh[i], body + S * (size_t)i, S);
        lens[i] = S;
      }
    }
    uint8_t* out = NULL;
    CHECK(rs_host_alloc(ctx, L, (void**)&out) == RS_OK);
    CHECK(rs_codec_decode(ctx, k, m, sh, lens, out, (int64_t)L) == RS_OK);
    CHECK(memcmp(out, body, L) == 0);
    for (int i = 0; i < n; i++) {
      CHECK(lens[i] == S && memcmp(sh[i], body + S * (size_t)i, S) == 0);
      CHECK(rs_host_free(ctx, sh[i]) == RS_OK);
    }
    CHECK(rs_host_free(ctx, out) == RS_OK);
    CHECK(rs_host_free(ctx, body) == RS_OK);
    CHECK(rs_host_free(ctx, body) == RS_E_ARG); /* already freed */
    CHECK(rs_host_free(ctx, want) == RS_E_ARG); /* not rs_host_alloc memory */
    free(lens); free(sh); free(want); free(pout); free(din);
  }
}

int main(int argc, char** argv) {
  const int need_gpu = argc > 1 && strcmp(argv[1], "gpu") == 0;
  rs_ctx* ctx = NULL;
  const int rc = rs_init(&ctx, 0);
  if (rc == RS_E_HIP && !need_gpu) {
    /* No device: a stand-in handle; these paths must return before touching it. */
    static char opaque[64];
    const int k = 4, m = 2;
    const size_t S = 1000;
    uint8_t* sh[6];
    for (int i = 0; i < 6; i++) {
      sh[i] = (uint8_t*)malloc(S);
      memset(sh[i], i, S);
    }
    argument_paths((rs_ctx*)opaque, k, m, S, sh);
    for (int i = 0; i < 6; i++) free(sh[i]);
    printf(fails ? "cgo_drive FAILED (%d)\n" : "cgo_drive ok (argument paths, no device)\n", fails);
    return fails != 0;
  }
  if (rc != RS_OK) {
    printf("rs_init failed: %s\n", rs_strerror(rc));
    return 2;
  }
  device_paths(ctx, 4, 2, 2);                /* "hi": S = 1 */
  device_paths(ctx, 10, 4, (1u << 20) + 7);  /* ragged tail */
  device_paths(ctx, 4, 2, 3u << 20);         /* RS(4,2) 1 MiB shards */
  device_paths(ctx, 16, 4, 64u << 20);       /* pipeline with several chunks */
  host_body_paths(ctx, 10, 4, (10u << 20) + 3, 1); /* pinned bodies, zero-copy */
  host_body_paths(ctx, 4, 2, 4096, 0);             /* a small body: the one-dispatch path */
  rs_shutdown(ctx);
  printf(fails ? "cgo_drive FAILED (%d)\n" : "cgo_drive ok (device round trips)\n", fails);
  return fails != 0;
}
