/* Per-call encode rate of the CPU port of upstream's SIMD codec (development tool).
 *
 * Calls oracle/rs_oracle.c orc_apply_simd (GFNI, byte ranges on a persistent thread
 * pool, like upstream codeSomeShardsP) once per object: the m parity shards of k data
 * shards that alias the object, as upstream Split leaves them. Paired with
 * `CALLFS_E2E_ENCODER=1 tools/e2e_native` (the GPU path the cgo shim takes) it locates
 * the object size above which the shim should hand a request to the GPU (INTEGRATION.md,
 * CALLFS_ERASURE__GPU_MIN_BYTES).
 *
 * build: gcc -O2 tests/perf/cpu_port_native.c -Loracle/build -lrs_oracle \
 *          -Wl,-rpath,'$ORIGIN/../../oracle/build' -o tests/perf/cpu_port_native
 * run:   tests/perf/cpu_port_native k m object_bytes threads seconds
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

int orc_encode_matrix(int k, int m, uint8_t* out);
void orc_apply_simd(int rows, int k, const uint8_t* coef, size_t S, const uint8_t* const* in,
                    uint8_t* const* out, int nthreads);

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: %s k m object_bytes threads seconds\n", argv[0]);
    return 2;
  }
  const int k = atoi(argv[1]), m = atoi(argv[2]), th = atoi(argv[4]);
  const size_t L = strtoull(argv[3], NULL, 0);
  const double secs = atof(argv[5]);
  if (k < 1 || m < 1 || k + m > 256 || L == 0) return 2;
  const size_t S = (L + k - 1) / k;
  uint8_t* E = malloc((size_t)(k + m) * k);
  if (orc_encode_matrix(k, m, E)) return 1;
  uint8_t* obj = malloc(S * k);
  uint8_t* par = malloc(S * m);
  for (size_t i = 0; i < S * k; i++) obj[i] = (uint8_t)(i * 2654435761u >> 13);
  const uint8_t* in[256];
  uint8_t* out[256];
  for (int i = 0; i < k; i++) in[i] = obj + S * i;
  for (int j = 0; j < m; j++) out[j] = par + S * j;
  orc_apply_simd(m, k, E + (size_t)k * k, S, in, out, th); /* warm: pool threads, caches */
  long n = 0;
  const double t0 = now();
  double t1;
  do {
    orc_apply_simd(m, k, E + (size_t)k * k, S, in, out, th);
    n++;
  } while ((t1 = now()) - t0 < secs);
  printf("{\"api\": \"cpu-port\", \"k\": %d, \"m\": %d, \"object_bytes\": %zu, \"threads\": %d, "
         "\"encode_gib_s\": %.3f, \"us_per_call\": %.1f}\n",
         k, m, L, th, n * (double)L / (t1 - t0) / 1073741824.0, (t1 - t0) / n * 1e6);
  free(E);
  free(obj);
  free(par);
  return 0;
}
