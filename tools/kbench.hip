// Kernel A/B harness for the RS vector kernel (development tool, not product).
//
// Interleaves every variant in one process (cdna_hip_programming.md §5.4 rule 24):
// R rounds x V variants, each timed with hipEvents over ITERS back-to-back launches on
// one stream, on a device-resident batch far larger than the 256 MiB MALL. Every
// variant's parity is compared with the production policy's (bit-exact). Also times
// an XOR-only kernel with the identical access pattern (K loads + R stores per 16-B
// vector, no GF work) as the memory ceiling of this traffic shape, and hipMemcpy D2D.
//
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I callfs_amd/csrc tools/kbench.hip \
//          callfs_amd/csrc/rs_kernels.hip -o tools/kbench
// run:   tools/kbench [k m shard_bytes stripes rounds iters]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "gf256.hpp"
#include "rs_apply.hpp"
#include "rs_kernels.hpp"

using namespace callfs;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,            \
                   hipGetErrorString(e_));                                      \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

__global__ void fill_kernel(uint32_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = static_cast<uint32_t>(i) * 0x9E3779B1u ^ seed ^ static_cast<uint32_t>(i >> 32);
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    p[i] = x;
  }
}

// Memory ceiling for this traffic shape: K 16-B loads, R 16-B stores per lane.
template <int K, int R, bool NT>
__global__ __launch_bounds__(256) void xor_stream(ApplyArgs a) {
  using P = dev::Policy<4, 1, NT, NT, false>;
  const uint32_t tps = static_cast<uint32_t>((a.nvec + 255) / 256);
  const uint32_t t = blockIdx.x;
  const uint32_t stripe = t / tps;
  const uint64_t v = static_cast<uint64_t>(t - stripe * tps) * 256 + threadIdx.x;
  if (v >= a.nvec) return;
  dev::cptr<const uint8_t*> in = dev::as_const(a.in_tab) + static_cast<size_t>(stripe) * K;
  dev::cptr<uint8_t*> out = dev::as_const(a.out_tab) + static_cast<size_t>(stripe) * R;
  uint4 x[K];
#pragma unroll
  for (int i = 0; i < K; ++i) x[i] = dev::load16<P>(reinterpret_cast<const uint4*>(in[i]) + v);
  uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int i = 0; i < K; ++i) {
    acc.x ^= x[i].x; acc.y ^= x[i].y; acc.z ^= x[i].z; acc.w ^= x[i].w;
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
    dev::store16<P>(reinterpret_cast<uint4*>(out[r]) + v, make_uint4(acc.x + r, acc.y, acc.z, acc.w));
}


// Hybrid row split (VERDICT r03 item 3 probe): rows 0..RL-1 of a wide launch group take the
// LDS nibble tables with 8-byte entries (ds_read_b64, 2 LDS-array cycles per lookup where
// 16-byte entries take 4), rows RL..RL+RV-1 the v_perm products of the k <= 3 kernel
// (coefficient tables through the constant address space, s_load). Halves the LDS-array
// cycles of R = 16 and moves the rest onto the VALU. Consecutive tiles, ring of three.
template <int RL, int RV>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 8)))
void hybrid_kernel(ApplyArgs a, const uint8_t* ltabs8) {
  using namespace dev;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int K = a.K;
  {
    const uint4* src = reinterpret_cast<const uint4*>(ltabs8);
    uint4* dst = reinterpret_cast<uint4*>(smem);
    for (int j = threadIdx.x; j < K * 16; j += 512) dst[j] = src[j];
  }
  __syncthreads();
  const uint32_t lds0 = static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)smem));
  const uint32_t tps = static_cast<uint32_t>((a.nvec + 511) / 512);
  const uint32_t stripe = blockIdx.x / tps, tile = blockIdx.x - stripe * tps;
  const uint64_t v0 = static_cast<uint64_t>(tile) * 512 + threadIdx.x;
  if (v0 >= a.nvec) return;
  cptr<const uint8_t*> in = as_const(a.in_tab) + static_cast<size_t>(stripe) * K;
  cptr<uint8_t*> out = as_const(a.out_tab) + static_cast<size_t>(stripe) * a.R;
  const cptr<uint32_t> tabs = as_const(a.tabs);
  using P = Policy<2, 1, true, true, false, 512>;
  auto ld = [&](int i) { return load16<P>(reinterpret_cast<const uint4*>(in[i]) + v0); };
  typename LdsAcc<8>::T accL[4][4];
  uint32_t accV[RV][4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
#pragma unroll
    for (int j = 0; j < 4; ++j) accL[w][j] = 0;
#pragma unroll
    for (int r = 0; r < RV; ++r) accV[r][w] = 0;
  }
  uint4 x0 = ld(0), x1 = K > 1 ? ld(1) : x0, x2 = x0;
#pragma unroll 1
  for (int i = 0; i < K; ++i) {
    if (i + 2 < K) x2 = ld(i + 2);
    lds_mac<8>(accL, x0, lds0 + static_cast<uint32_t>(i) * 256u);
    const cptr<uint32_t> t = tabs + (static_cast<size_t>(i) * a.R + RL) * 5;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const Sel sel = selectors(word(x0, w));
#pragma unroll
      for (int r = 0; r < RV; ++r) accV[r][w] = fma1(accV[r][w], gf_mul4(sel, t + r * 5));
    }
    x0 = x1;
    x1 = x2;
  }
#pragma unroll
  for (int r = 0; r < RL; ++r)
    store16<P>(reinterpret_cast<uint4*>(out[r]) + v0,
               make_uint4(lds_row<8>(accL[0], r), lds_row<8>(accL[1], r), lds_row<8>(accL[2], r),
                          lds_row<8>(accL[3], r)));
#pragma unroll
  for (int r = 0; r < RV; ++r)
    store16<P>(reinterpret_cast<uint4*>(out[RL + r]) + v0,
               make_uint4(accV[r][0], accV[r][1], accV[r][2], accV[r][3]));
}

template <int R, class P>
void launch_lds(const ApplyArgs& a, hipStream_t s) {
  const unsigned g = dev::vec_grid<P>(a.nvec, a.batch);
  hipLaunchKernelGGL((dev::rs_apply_lds<R, P>), dim3(g), dim3(P::BS), dev::lds_bytes(a.K, R), s, a);
}

// Read-only ceiling: the K input streams, nothing stored unless an impossible value.
template <int K>
__global__ __launch_bounds__(512) void read_stream(ApplyArgs a) {
  using P = dev::Policy<4, 1, true, true, false>;
  const uint32_t tps = static_cast<uint32_t>((a.nvec + 511) / 512);
  const uint32_t t = blockIdx.x, stripe = t / tps;
  const uint64_t v = static_cast<uint64_t>(t - stripe * tps) * 512 + threadIdx.x;
  if (v >= a.nvec) return;
  dev::cptr<const uint8_t*> in = dev::as_const(a.in_tab) + static_cast<size_t>(stripe) * K;
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const uint4 x = dev::load16<P>(reinterpret_cast<const uint4*>(in[i]) + v);
    acc ^= x.x ^ x.y ^ x.z ^ x.w;
  }
  if (acc == 0x9E3779B9u && v == 12345) *a.status = 1;
}

// Write-only ceiling: R output streams of a register value.
template <int R>
__global__ __launch_bounds__(512) void write_stream(ApplyArgs a) {
  using P = dev::Policy<4, 1, true, true, false>;
  const uint32_t tps = static_cast<uint32_t>((a.nvec + 511) / 512);
  const uint32_t t = blockIdx.x, stripe = t / tps;
  const uint64_t v = static_cast<uint64_t>(t - stripe * tps) * 512 + threadIdx.x;
  if (v >= a.nvec) return;
  dev::cptr<uint8_t*> out = dev::as_const(a.out_tab) + static_cast<size_t>(stripe) * R;
#pragma unroll
  for (int r = 0; r < R; ++r)
    dev::store16<P>(reinterpret_cast<uint4*>(out[r]) + v, make_uint4(t, r, 7, 9));
}

// Read probe: every shard stream of the layout (K inputs and the R output slots) read in
// tile order ORD, nothing stored unless an impossible value -- a side-effect-free
// stand-in for the kernel's access pattern (does its ranking of tile orders match the
// kernel's?).
template <int ORD>
__global__ __launch_bounds__(512) void read_probe(ApplyArgs a) {
  const uint32_t tps = static_cast<uint32_t>((a.nvec + 511) / 512);
  uint32_t stripe, tile;
  map_tile<ORD>(blockIdx.x, tps, static_cast<uint32_t>(a.batch), stripe, tile);
  const uint64_t v = static_cast<uint64_t>(tile) * 512 + threadIdx.x;
  if (v >= a.nvec) return;
  using P = dev::Policy<4, 1, true, true, false>;
  dev::cptr<const uint8_t*> in = dev::as_const(a.in_tab) + static_cast<size_t>(stripe) * a.K;
  dev::cptr<uint8_t*> out = dev::as_const(a.out_tab) + static_cast<size_t>(stripe) * a.R;
  uint32_t acc = 0;
  for (int i = 0; i < a.K; ++i) {
    const uint4 x = dev::load16<P>(reinterpret_cast<const uint4*>(in[i]) + v);
    acc ^= x.x ^ x.y ^ x.z ^ x.w;
  }
  for (int r = 0; r < a.R; ++r) {
    const uint4 x = dev::load16<P>(reinterpret_cast<const uint4*>(out[r]) + v);
    acc ^= x.x ^ x.y ^ x.z ^ x.w;
  }
  if (acc == 0x9E3779B9u && v == 12345) *a.status = 1;
}

struct Variant {
  std::string name;
  std::function<void(const ApplyArgs&, hipStream_t)> launch;
  bool check = true;
};

template <int K, int R, class P>
Variant make_variant(const char* name, int blocks_per_cu = 8) {
  return Variant{name, [blocks_per_cu](const ApplyArgs& a, hipStream_t s) {
                   const unsigned g = dev::vec_grid<P>(a.nvec, a.batch, blocks_per_cu);
                   hipLaunchKernelGGL((dev::rs_apply_vec<K, R, P>), dim3(g), dim3(P::BS), 0, s, a);
                 }};
}

int main(int argc, char** argv) {
  const int k = argc > 1 ? std::atoi(argv[1]) : 10;
  const int m = argc > 2 ? std::atoi(argv[2]) : 4;
  const size_t S = argc > 3 ? std::strtoull(argv[3], nullptr, 0) : (1u << 20);
  const int B = argc > 4 ? std::atoi(argv[4]) : 256;
  const int rounds = argc > 5 ? std::atoi(argv[5]) : 5;
  const int iters = argc > 6 ? std::atoi(argv[6]) : 10;
  const size_t palign = argc > 7 ? std::strtoull(argv[7], nullptr, 0) : 256;
  const size_t ppad = argc > 8 ? std::strtoull(argv[8], nullptr, 0) : 0;  // extra bytes per shard
  if (m < 1 || m > 16 || k < 1 || k > 256) {
    std::fprintf(stderr, "need 1<=m<=16, 1<=k<=256\n");
    return 2;
  }
  const int n = k + m;
  const size_t pitch = (S + palign - 1) / palign * palign + ppad;
  const size_t total = pitch * n * B;
  uint8_t* buf;
  CK(hipMalloc(&buf, total));
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(buf),
                     total / 4, 12345u);
  // KB_OUT_SEP=1: output rows in a separate buffer at a 256-B-aligned pitch (inputs keep
  // `pitch`); KB_IN_SEP=1: input rows there instead (unaligned-shard A/B: which side
  // pays for misaligned 16-B accesses)
  const bool out_sep = std::getenv("KB_OUT_SEP") != nullptr, in_sep = std::getenv("KB_IN_SEP") != nullptr;
  const size_t apitch = (S + 255) / 256 * 256;
  const size_t opitch = out_sep ? apitch : pitch;
  uint8_t* sep = nullptr;
  if (out_sep || in_sep) CK(hipMalloc(&sep, apitch * (out_sep ? m : k) * B));
  if (sep) hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(sep),
                              apitch * (out_sep ? m : k) * B / 4, 777u);
  uint8_t* ref;  // parity of the production variant
  CK(hipMalloc(&ref, opitch * m * B));

  // tables (encode: parity rows of E)
  Mat E;
  encode_matrix(k, m, E);
  std::vector<uint32_t> tabs(static_cast<size_t>(k) * m * 5);
  for (int i = 0; i < k; ++i)
    for (int r = 0; r < m; ++r) perm_tables(E.at(k + r, i), &tabs[(static_cast<size_t>(i) * m + r) * 5]);
  const size_t lper = 32u * nibble_width(m);
  std::vector<uint8_t> ltabs(static_cast<size_t>(k) * lper);
  for (int i = 0; i < k; ++i) {
    uint8_t col[16] = {0};
    for (int r = 0; r < m && r < 16; ++r) col[r] = E.at(k + r, i);
    nibble_tables(col, m, &ltabs[static_cast<size_t>(i) * lper]);
  }
  std::vector<const uint8_t*> in(static_cast<size_t>(B) * k);
  std::vector<uint8_t*> out(static_cast<size_t>(B) * m);
  // KB_IN / KB_OUT: comma lists of the stripe slots read / written (a decode pattern's
  // shard placement); default slots 0..k-1 in, k..n-1 out
  std::vector<int> islot(k), oslot(m);
  for (int i = 0; i < k; ++i) islot[i] = i;
  for (int r = 0; r < m; ++r) oslot[r] = k + r;
  auto parse = [](const char* e, std::vector<int>& v) {
    if (!e) return;
    std::string str(e);
    size_t p = 0;
    for (int& x : v) {
      x = std::atoi(str.c_str() + p);
      p = str.find(',', p);
      if (p == std::string::npos) break;
      ++p;
    }
  };
  parse(std::getenv("KB_IN"), islot);
  parse(std::getenv("KB_OUT"), oslot);
  for (int b = 0; b < B; ++b) {
    for (int i = 0; i < k; ++i)
      in[b * k + i] = in_sep ? sep + (static_cast<size_t>(b) * k + i) * apitch
                             : buf + (static_cast<size_t>(b) * n + islot[i]) * pitch;
    for (int r = 0; r < m; ++r)
      out[b * m + r] = out_sep ? sep + (static_cast<size_t>(b) * m + r) * apitch
                               : buf + (static_cast<size_t>(b) * n + oslot[r]) * pitch;
  }
  void *d_in, *d_out, *d_tabs, *d_ltabs;
  int* d_status;
  CK(hipMalloc(&d_in, in.size() * sizeof(void*)));
  CK(hipMalloc(&d_out, out.size() * sizeof(void*)));
  CK(hipMalloc(&d_tabs, tabs.size() * 4));
  CK(hipMalloc(&d_ltabs, ltabs.size()));
  CK(hipMemcpy(d_ltabs, ltabs.data(), ltabs.size(), hipMemcpyHostToDevice));
  CK(hipMalloc(&d_status, 4));
  CK(hipMemcpy(d_in, in.data(), in.size() * sizeof(void*), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_out, out.data(), out.size() * sizeof(void*), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_tabs, tabs.data(), tabs.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(d_status, 0, 4));
  // KB_HYBRID: 8-byte nibble tables of rows 0..7 (hybrid_kernel's LDS rows)
  static void* d_ltabs8 = nullptr;
  if (m > 8) {
    std::vector<uint8_t> l8(static_cast<size_t>(k) * 256);
    for (int i = 0; i < k; ++i) {
      uint8_t col[8];
      for (int r = 0; r < 8; ++r) col[r] = E.at(k + r, i);
      nibble_tables(col, 8, &l8[static_cast<size_t>(i) * 256]);
    }
    CK(hipMalloc(&d_ltabs8, l8.size()));
    CK(hipMemcpy(d_ltabs8, l8.data(), l8.size(), hipMemcpyHostToDevice));
  }

  ApplyArgs a{};
  a.in_tab = static_cast<const uint8_t* const*>(d_in);
  a.out_tab = static_cast<uint8_t* const*>(d_out);
  a.tabs = static_cast<const uint32_t*>(d_tabs);
  a.ltabs = static_cast<const uint8_t*>(d_ltabs);
  a.S = S;
  a.nvec = S / 16;
  a.verify_mask = 0;
  a.status = d_status;
  a.K = k;
  a.R = m;
  a.batch = B;
  {  // stripe 0's shard addresses, as rs_capi.cpp fill_meta computes it
    std::vector<const void*> s0(in.begin(), in.begin() + k);
    s0.insert(s0.end(), out.begin(), out.begin() + m);
    a.addr_tz = shard_addr_tz(s0.data(), k + m);
    a.stripe_stride = B > 1 ? static_cast<uint64_t>(pitch) * n : 0;
    a.in_misalign = 0;
    for (const uint8_t* p : in) a.in_misalign |= static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p)) & 15u;
    a.out_misalign = 0;
    for (uint8_t* p : out) a.out_misalign |= static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p)) & 15u;
  }

  using namespace dev;
  using Prod = Policy<4, 1, true, true, false, 512, 2, 0>;  // = rs_kernels.hip ProdPolicy
  std::vector<Variant> vs;
  // what the library runs for this (K, R): rs_kernels.hip launch_apply's dispatch
  vs.push_back(Variant{"prod dispatch", [](const ApplyArgs& a, hipStream_t s) {
                         CK(launch_apply(a, s));
                       }});
  if (std::getenv("KB_SLICE")) {  // the production dispatch at other launch-slice sizes
    static const int streams = k + m;
    auto sliced = [](const char* name, double gib) {
      return Variant{name, [gib](const ApplyArgs& a, hipStream_t s) {
                       set_slice_tiles_for_tuning(
                           gib <= 0 ? 0 : static_cast<long long>(gib * (1ull << 30) / (8192.0 * streams)));
                       CK(launch_apply(a, s));
                       set_slice_tiles_for_tuning(-1);
                     }};
    };
    vs.push_back(sliced("prod slice none", 0));
    vs.push_back(sliced("prod slice 1GiB", 1));
    vs.push_back(sliced("prod slice 4GiB", 4));
    vs.push_back(sliced("prod slice 8GiB", 8));
  }
  if (const char* sp = std::getenv("KB_SPLIT")) {  // same work as launches over B/N stripes each
    static const int parts = std::max(1, std::atoi(sp));
    vs.push_back(Variant{"prod split", [](const ApplyArgs& a, hipStream_t s) {
                           const int per = (a.batch + parts - 1) / parts;
                           for (int b0 = 0; b0 < a.batch; b0 += per) {
                             ApplyArgs p = a;
                             p.batch = std::min(per, a.batch - b0);
                             p.in_tab = a.in_tab + static_cast<size_t>(b0) * a.K;
                             p.out_tab = a.out_tab + static_cast<size_t>(b0) * a.R;
                             CK(launch_apply(p, s));
                           }
                         }});
  }
  if (std::getenv("KB_BYTES"))  // the byte kernel over the whole shard (unaligned-pointer dispatch)
    vs.push_back(Variant{"byte-kernel dispatch", [](const ApplyArgs& a, hipStream_t s) {
                           CK(launch_apply(a, s, /*bytes_only=*/true));
                         }});
  switch (m) {  // v_perm kernel (runtime K) for this row count
    case 1: vs.push_back(make_variant<0, 1, Prod>("prod rtK nt")); break;
    case 2: vs.push_back(make_variant<0, 2, Prod>("prod rtK nt")); break;
    case 3: vs.push_back(make_variant<0, 3, Prod>("prod rtK nt")); break;
    case 4: vs.push_back(make_variant<0, 4, Prod>("prod rtK nt")); break;
    case 5: vs.push_back(make_variant<0, 5, Prod>("prod rtK nt")); break;
    case 6: vs.push_back(make_variant<0, 6, Prod>("prod rtK nt")); break;
    case 7: vs.push_back(make_variant<0, 7, Prod>("prod rtK nt")); break;
    case 8: vs.push_back(make_variant<0, 8, Prod>("prod rtK nt")); break;
  }
  const bool rs10_4 = k == 10 && m == 4;
  using L512 = Policy<4, 1, true, true, false, 512, 2, 0>;
  using L256 = Policy<4, 1, true, true, false, 256, 2, 0>;
  using L512w2 = Policy<2, 1, true, true, false, 512, 2, 0>;
  switch (m) {
    case 4:
      vs.push_back(Variant{"lds bs512", [](const ApplyArgs& a, hipStream_t s) { launch_lds<4, L512>(a, s); }});
      vs.push_back(Variant{"lds bs256", [](const ApplyArgs& a, hipStream_t s) { launch_lds<4, L256>(a, s); }});
      vs.push_back(Variant{"lds bs512 wpe2", [](const ApplyArgs& a, hipStream_t s) { launch_lds<4, L512w2>(a, s); }});
      break;
    case 8:
      vs.push_back(Variant{"lds bs512 (prod R>=5)", [](const ApplyArgs& a, hipStream_t s) { launch_lds<8, L512w2>(a, s); }});
      vs.push_back(Variant{"lds bs512", [](const ApplyArgs& a, hipStream_t s) { launch_lds<8, L512>(a, s); }});
      vs.push_back(Variant{"lds bs256", [](const ApplyArgs& a, hipStream_t s) { launch_lds<8, L256>(a, s); }});
      vs.push_back(Variant{"lds bs512 wpe2", [](const ApplyArgs& a, hipStream_t s) { launch_lds<8, L512w2>(a, s); }});
      break;
    case 2:
      vs.push_back(Variant{"lds bs512", [](const ApplyArgs& a, hipStream_t s) { launch_lds<2, L512>(a, s); }});
      break;
    case 6:
      vs.push_back(Variant{"lds bs512", [](const ApplyArgs& a, hipStream_t s) { launch_lds<6, L512>(a, s); }});
      break;
    case 9: vs.push_back(Variant{"lds RT=9", [](const ApplyArgs& a, hipStream_t s) { launch_lds<9, L512w2>(a, s); }}); break;
    case 10: vs.push_back(Variant{"lds RT=10", [](const ApplyArgs& a, hipStream_t s) { launch_lds<10, L512w2>(a, s); }}); break;
    case 11: vs.push_back(Variant{"lds RT=11", [](const ApplyArgs& a, hipStream_t s) { launch_lds<11, L512w2>(a, s); }}); break;
    case 12: vs.push_back(Variant{"lds RT=12", [](const ApplyArgs& a, hipStream_t s) { launch_lds<12, L512w2>(a, s); }}); break;
    case 13: vs.push_back(Variant{"lds RT=13", [](const ApplyArgs& a, hipStream_t s) { launch_lds<13, L512w2>(a, s); }}); break;
    case 14: vs.push_back(Variant{"lds RT=14", [](const ApplyArgs& a, hipStream_t s) { launch_lds<14, L512w2>(a, s); }}); break;
    case 15: vs.push_back(Variant{"lds RT=15", [](const ApplyArgs& a, hipStream_t s) { launch_lds<15, L512w2>(a, s); }}); break;
    case 16:
      vs.push_back(Variant{"lds RT=16 direct", [](const ApplyArgs& a, hipStream_t s) { launch_lds<16, L512w2>(a, s); }});
      break;
  }
  if (m <= 4) {  // LDS kernel with the production LDS policy, for the R <= 4 dispatch choice
    static void (*const lds_r[4])(const ApplyArgs&, hipStream_t) = {
        launch_lds<1, L512w2>, launch_lds<2, L512w2>, launch_lds<3, L512w2>, launch_lds<4, L512w2>};
    vs.push_back(Variant{"lds prod-policy", [m](const ApplyArgs& a, hipStream_t s) { lds_r[m - 1](a, s); }});
  }
  if (k <= 3 && m <= 4 && std::getenv("KB_ORD")) {  // v_perm kernel tile orders (k <= 3)
#define KB_VORD(RT)                                                                                       \
  vs.push_back(make_variant<0, RT, Policy<4, 1, true, true, false, 512, 2, 0>>("vperm ord consec"));   \
  vs.push_back(make_variant<0, RT, Policy<4, 1, true, true, false, 512, 2, 2>>("vperm ord g8"));       \
  vs.push_back(make_variant<0, RT, Policy<4, 1, true, true, false, 512, 2, 5>>("vperm ord g2"));       \
  vs.push_back(make_variant<0, RT, Policy<4, 1, true, true, false, 512, 2, 6>>("vperm ord q8"));       \
  vs.push_back(make_variant<0, RT, Policy<4, 1, true, true, false, 512, 2, 8>>("vperm ord q16"));
    switch (m) {
      case 1: KB_VORD(1) break;
      case 2: KB_VORD(2) break;
      case 3: KB_VORD(3) break;
      case 4: KB_VORD(4) break;
    }
  }
  if ((m == 2 || m == 3 || m == 4 || m == 8) && std::getenv("KB_TRIDB")) {
    // triple-loop forms: WIX 2 (production), 4 (loads past K leave zeros), 3 (two register
    // sets, no conditional loads), 3 at <= 80 VGPRs, 5 (pairs in two register sets);
    // orders X32, G2, Q16
#define KB_TW(R, ORD, WX, WP) Policy<(WP), 1, true, true, false, 512, 2, ORD, 0, false, 0, false, 0, 0, WX>
#define KB_TV(R, ORD, WX, WP, NAME) \
  vs.push_back(Variant{NAME, [](const ApplyArgs& a, hipStream_t s) { launch_lds<R, KB_TW(R, ORD, WX, WP)>(a, s); }});
#define KB_TVS(R, WP8)                                                                            \
  KB_TV(R, 11, 2, WP8, "tri2 x32") KB_TV(R, 11, 4, WP8, "tri4 x32") KB_TV(R, 11, 3, 2, "tridb x32") \
  KB_TV(R, 11, 3, 6, "tridb6 x32") KB_TV(R, 5, 2, WP8, "tri2 g2") KB_TV(R, 5, 4, WP8, "tri4 g2")    \
  KB_TV(R, 5, 3, 2, "tridb g2") KB_TV(R, 8, 2, WP8, "tri2 q16") KB_TV(R, 8, 3, 2, "tridb q16")      \
  KB_TV(R, 11, 5, 2, "pairdb x32") KB_TV(R, 5, 5, 2, "pairdb g2")
    switch (m) {
      case 2: KB_TVS(2, 8) break;
      case 3: KB_TVS(3, 8) break;
      case 4: KB_TVS(4, 8) break;
      case 8: KB_TVS(8, 2) break;
    }
#undef KB_TVS
#undef KB_TV
#undef KB_TW
  }
  if (m <= 4 && std::getenv("KB_TRIORD")) {  // triple loads (WIX 2) in every tile order
#define KB_TP(ORD) Policy<8, 1, true, true, false, 512, 2, ORD, 0, false, 0, false, 0, 0, 2>
#define KB_TRI(RT, ORD, NAME) \
  vs.push_back(Variant{NAME, [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, KB_TP(ORD)>(a, s); }});
#define KB_TRIS(RT) KB_TRI(RT, 0, "tri ord consec") KB_TRI(RT, 2, "tri ord g8") KB_TRI(RT, 4, "tri ord g4") \
  KB_TRI(RT, 5, "tri ord g2") KB_TRI(RT, 6, "tri ord q8") KB_TRI(RT, 7, "tri ord q32") KB_TRI(RT, 8, "tri ord q16") \
  KB_TRI(RT, 9, "tri ord q64") KB_TRI(RT, 10, "tri ord x8") KB_TRI(RT, 11, "tri ord x32")
    switch (m) {
      case 1: KB_TRIS(1) break;
      case 2: KB_TRIS(2) break;
      case 3: KB_TRIS(3) break;
      case 4: KB_TRIS(4) break;
    }
#undef KB_TRIS
#undef KB_TRI
#undef KB_TP
  }
  if ((m == 2 || m == 3 || m == 4 || m == 8) && std::getenv("KB_ORD")) {  // LDS kernel tile orders
    using O0 = Policy<2, 1, true, true, false, 512, 2, 0>;
    using O2 = Policy<2, 1, true, true, false, 512, 2, 2>;
    using O3 = Policy<2, 1, true, true, false, 512, 2, 3>;
    using O4 = Policy<2, 1, true, true, false, 512, 2, 4>;
    using O5 = Policy<2, 1, true, true, false, 512, 2, 5>;
    using O6 = Policy<2, 1, true, true, false, 512, 2, 6>;
    using O7 = Policy<2, 1, true, true, false, 512, 2, 7>;
    using O8 = Policy<2, 1, true, true, false, 512, 2, 8>;
    using O9 = Policy<2, 1, true, true, false, 512, 2, 9>;
#define KB_ORDS(RT)                                                                                  \
  vs.push_back(Variant{"lds ord consec", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, O0>(a, s); }}); \
  vs.push_back(Variant{"lds ord g8", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, O2>(a, s); }}); \
  vs.push_back(Variant{"lds ord g32", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, O3>(a, s); }}); \
  vs.push_back(Variant{"lds ord g4", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, O4>(a, s); }}); \
  vs.push_back(Variant{"lds ord g2", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, O5>(a, s); }}); \
  vs.push_back(Variant{"lds ord q8", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, O6>(a, s); }}); \
  vs.push_back(Variant{"lds ord q32", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, O7>(a, s); }}); \
  vs.push_back(Variant{"lds ord q16", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, O8>(a, s); }}); \
  vs.push_back(Variant{"lds ord q64", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, O9>(a, s); }});
    switch (m) {
      case 2: KB_ORDS(2) break;
      case 3: KB_ORDS(3) break;
      case 4: KB_ORDS(4) break;
      case 8: KB_ORDS(8) break;
    }
  }
  if (std::getenv("KB_ORD") && m > 8) {  // tile orders for wider row groups (R 9..16)
    using W0 = Policy<2, 1, true, true, false, 512, 4, 0, 1>;  // = rs_kernels.hip LdsWidePolicy
    using W2 = Policy<2, 1, true, true, false, 512, 4, 5, 1>;
    using W8 = Policy<2, 1, true, true, false, 512, 4, 2, 1>;
    using WQ = Policy<2, 1, true, true, false, 512, 4, 6, 1>;
#define KB_WORD(RT, P0)                                                                           \
  vs.push_back(Variant{"lds ord consecutive", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, P0>(a, s); }}); \
  vs.push_back(Variant{"lds ord wide g2", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, W2>(a, s); }}); \
  vs.push_back(Variant{"lds ord wide g8", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, W8>(a, s); }}); \
  vs.push_back(Variant{"lds ord wide q8", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, WQ>(a, s); }});
    switch (m) {
      case 12: KB_WORD(12, W0) break;
      case 16: KB_WORD(16, W0) break;
    }
  }
  if (std::getenv("KB_PROBE")) {  // read probes in each tile order (bytes: all n streams)
#define KB_PROBE_V(NAME, ORD)                                                                  \
  vs.push_back(Variant{NAME, [](const ApplyArgs& a, hipStream_t s) {                           \
                         const unsigned g = static_cast<unsigned>((a.nvec + 511) / 512 * a.batch); \
                         hipLaunchKernelGGL((read_probe<ORD>), dim3(g), dim3(512), 0, s, a);  \
                       }, false});
    KB_PROBE_V("probe c", 0) KB_PROBE_V("probe g8", 2) KB_PROBE_V("probe g2", 5)
    KB_PROBE_V("probe q8", 6) KB_PROBE_V("probe q16", 8) KB_PROBE_V("probe q64", 9)
  }
  if (std::getenv("KB_RING")) {  // unrolled input ring of PD+1 slots (RING = 1)
    using R2 = Policy<2, 1, true, true, false, 512, 2, 0, 1>;
    using R3 = Policy<2, 1, true, true, false, 512, 3, 0, 1>;
    using R4 = Policy<2, 1, true, true, false, 512, 4, 0, 1>;
    using R6 = Policy<2, 1, true, true, false, 512, 6, 0, 1>;
#define KB_RINGS(RT)                                                                                    \
  vs.push_back(Variant{"lds ring pd2", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, R2>(a, s); }}); \
  vs.push_back(Variant{"lds ring pd3", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, R3>(a, s); }}); \
  vs.push_back(Variant{"lds ring pd4", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, R4>(a, s); }}); \
  vs.push_back(Variant{"lds ring pd6", [](const ApplyArgs& a, hipStream_t s) { launch_lds<RT, R6>(a, s); }});
    switch (m) {
      case 4: KB_RINGS(4) break;
      case 8: KB_RINGS(8) break;
      case 12: KB_RINGS(12) break;
      case 16: KB_RINGS(16) break;
    }
  }
  if (std::getenv("KB_REALIGN")) {  // aligned loads + in-register realignment (misaligned inputs)
    static void (*const ra[8])(const ApplyArgs&, hipStream_t) = {
#define KB_RA(R) [](const ApplyArgs& a, hipStream_t s) { launch_lds<R, Policy<2, 1, true, true, false, 512, 2, 5, 0, false, true>>(a, s); }
        KB_RA(1), KB_RA(2), KB_RA(3), KB_RA(4), KB_RA(5), KB_RA(6), KB_RA(7), KB_RA(8)};
#undef KB_RA
    static void (*const rc[8])(const ApplyArgs&, hipStream_t) = {
#define KB_RA(R) [](const ApplyArgs& a, hipStream_t s) { launch_lds<R, Policy<2, 1, true, true, false, 512, 2, 0, 0, false, true>>(a, s); }
        KB_RA(1), KB_RA(2), KB_RA(3), KB_RA(4), KB_RA(5), KB_RA(6), KB_RA(7), KB_RA(8)};
#undef KB_RA
    if (m <= 8) {
      vs.push_back(Variant{"realign g2", [m](const ApplyArgs& a, hipStream_t s) { ra[m - 1](a, s); }});
      vs.push_back(Variant{"realign consec", [m](const ApplyArgs& a, hipStream_t s) { rc[m - 1](a, s); }});
    }
  }
  if (std::getenv("KB_SDWA")) {  // table addresses by v_or_b32_sdwa instead of v_perm_b32
#define KB_SDP(R, ORD, SD) Policy<2, 1, true, true, false, 512, (R > 8 ? 4 : 2), ORD, (R > 8 ? 1 : 0), false, false, SD>
#define KB_SD(R) [](const ApplyArgs& a, hipStream_t s) { launch_lds<R, KB_SDP(R, 5, true)>(a, s); }
    static void (*const sd_g2[16])(const ApplyArgs&, hipStream_t) = {
        KB_SD(1), KB_SD(2), KB_SD(3), KB_SD(4), KB_SD(5), KB_SD(6), KB_SD(7), KB_SD(8),
        KB_SD(9), KB_SD(10), KB_SD(11), KB_SD(12), KB_SD(13), KB_SD(14), KB_SD(15), KB_SD(16)};
#undef KB_SD
#define KB_SD(R) [](const ApplyArgs& a, hipStream_t s) { launch_lds<R, KB_SDP(R, 0, true)>(a, s); }
    static void (*const sd_c[16])(const ApplyArgs&, hipStream_t) = {
        KB_SD(1), KB_SD(2), KB_SD(3), KB_SD(4), KB_SD(5), KB_SD(6), KB_SD(7), KB_SD(8),
        KB_SD(9), KB_SD(10), KB_SD(11), KB_SD(12), KB_SD(13), KB_SD(14), KB_SD(15), KB_SD(16)};
#undef KB_SD
#define KB_SD(R) [](const ApplyArgs& a, hipStream_t s) { launch_lds<R, KB_SDP(R, 5, false)>(a, s); }
    static void (*const pm_g2[16])(const ApplyArgs&, hipStream_t) = {
        KB_SD(1), KB_SD(2), KB_SD(3), KB_SD(4), KB_SD(5), KB_SD(6), KB_SD(7), KB_SD(8),
        KB_SD(9), KB_SD(10), KB_SD(11), KB_SD(12), KB_SD(13), KB_SD(14), KB_SD(15), KB_SD(16)};
#undef KB_SD
#define KB_SD(R) [](const ApplyArgs& a, hipStream_t s) { launch_lds<R, KB_SDP(R, 0, false)>(a, s); }
    static void (*const pm_c[16])(const ApplyArgs&, hipStream_t) = {
        KB_SD(1), KB_SD(2), KB_SD(3), KB_SD(4), KB_SD(5), KB_SD(6), KB_SD(7), KB_SD(8),
        KB_SD(9), KB_SD(10), KB_SD(11), KB_SD(12), KB_SD(13), KB_SD(14), KB_SD(15), KB_SD(16)};
#undef KB_SD
#undef KB_SDP
    vs.push_back(Variant{"sdwa g2", [m](const ApplyArgs& a, hipStream_t s) { sd_g2[m - 1](a, s); }});
    vs.push_back(Variant{"perm g2", [m](const ApplyArgs& a, hipStream_t s) { pm_g2[m - 1](a, s); }});
    vs.push_back(Variant{"sdwa consec", [m](const ApplyArgs& a, hipStream_t s) { sd_c[m - 1](a, s); }});
    vs.push_back(Variant{"perm consec", [m](const ApplyArgs& a, hipStream_t s) { pm_c[m - 1](a, s); }});
  }
  if (std::getenv("KB_HYBRID") && (m == 12 || m == 16)) {  // LDS rows 0..7 + v_perm rows 8..m-1
    auto hv = [](const ApplyArgs& a, hipStream_t s) {
      const unsigned g = static_cast<unsigned>((a.nvec + 511) / 512 * a.batch);
      const size_t lds = static_cast<size_t>(a.K) * 256;
      if (a.R == 16)
        hipLaunchKernelGGL((hybrid_kernel<8, 8>), dim3(g), dim3(512), lds, s, a,
                           static_cast<const uint8_t*>(d_ltabs8));
      else
        hipLaunchKernelGGL((hybrid_kernel<8, 4>), dim3(g), dim3(512), lds, s, a,
                           static_cast<const uint8_t*>(d_ltabs8));
    };
    if (std::getenv("KB_HYBRID_FIRST")) vs.insert(vs.begin(), Variant{"hybrid 8+v", hv});
    else vs.push_back(Variant{"hybrid 8+v", hv});
  }
  if (std::getenv("KB_PROD2"))  // the production dispatch again, at another place in the order
    vs.push_back(Variant{"prod dispatch (2nd)", [](const ApplyArgs& a, hipStream_t s) {
                           CK(launch_apply(a, s));
                         }});
  if (std::getenv("KB_PROBE63") && m <= 8) {  // wave-tiling probes (lane 63 idle; parity incomplete)
    static void (*const p1[8])(const ApplyArgs&, hipStream_t) = {
#define KB_P(R) [](const ApplyArgs& a, hipStream_t s) { launch_lds<R, Policy<2, 1, true, true, false, 512, 2, 0, 0, false, false, false, 1>>(a, s); }
        KB_P(1), KB_P(2), KB_P(3), KB_P(4), KB_P(5), KB_P(6), KB_P(7), KB_P(8)};
#undef KB_P
    static void (*const p2[8])(const ApplyArgs&, hipStream_t) = {
#define KB_P(R) [](const ApplyArgs& a, hipStream_t s) { launch_lds<R, Policy<2, 1, true, true, false, 512, 2, 0, 0, false, false, false, 2>>(a, s); }
        KB_P(1), KB_P(2), KB_P(3), KB_P(4), KB_P(5), KB_P(6), KB_P(7), KB_P(8)};
#undef KB_P
    static void (*const rc[8])(const ApplyArgs&, hipStream_t) = {
#define KB_P(R) [](const ApplyArgs& a, hipStream_t s) { launch_lds<R, Policy<2, 1, true, true, false, 512, 2, 0, 0, false, true>>(a, s); }
        KB_P(1), KB_P(2), KB_P(3), KB_P(4), KB_P(5), KB_P(6), KB_P(7), KB_P(8)};
#undef KB_P
    vs.push_back(Variant{"probe 63-vec waves", [m](const ApplyArgs& a, hipStream_t s) { p1[m - 1](a, s); }, false});
    vs.push_back(Variant{"probe 64-vec waves lane63 idle", [m](const ApplyArgs& a, hipStream_t s) { p2[m - 1](a, s); }, false});
    vs.push_back(Variant{"realign consec", [m](const ApplyArgs& a, hipStream_t s) { rc[m - 1](a, s); }});
    static void (*const ro[8])(const ApplyArgs&, hipStream_t) = {
#define KB_P(R) [](const ApplyArgs& a, hipStream_t s) { ApplyArgs b = a; b.tail_in_vec = 1; launch_lds<R, Policy<(R <= 4 ? 8 : 2), 1, true, true, false, 512, 2, 0, 0, false, 2>>(b, s); }
        KB_P(1), KB_P(2), KB_P(3), KB_P(4), KB_P(5), KB_P(6), KB_P(7), KB_P(8)};
#undef KB_P
    vs.push_back(Variant{"realign out (loads+stores)", [m](const ApplyArgs& a, hipStream_t s) { ro[m - 1](a, s); }});
    vs.push_back(Variant{"plain consec", [m](const ApplyArgs& a, hipStream_t s) {
                           if (m == 4) launch_lds<4, Policy<2, 1, true, true, false, 512, 2, 0>>(a, s);
                           else if (m == 8) launch_lds<8, Policy<2, 1, true, true, false, 512, 2, 0>>(a, s);
                           else if (m == 2) launch_lds<2, Policy<2, 1, true, true, false, 512, 2, 0>>(a, s);
                         }});
  }
  {  // memory ceiling of this traffic shape: the LDS kernel's loads/stores/grid, no lookups
    static void (*const nomath_g2[16])(const ApplyArgs&, hipStream_t) = {
#define KB_NM(R) [](const ApplyArgs& a, hipStream_t s) { launch_lds<R, Policy<2, 1, true, true, false, 512, (R > 8 ? 4 : 2), 5, (R > 8 ? 1 : 0), true>>(a, s); }
        KB_NM(1), KB_NM(2), KB_NM(3), KB_NM(4), KB_NM(5), KB_NM(6), KB_NM(7), KB_NM(8),
        KB_NM(9), KB_NM(10), KB_NM(11), KB_NM(12), KB_NM(13), KB_NM(14), KB_NM(15), KB_NM(16)};
#undef KB_NM
    static void (*const nomath_c[16])(const ApplyArgs&, hipStream_t) = {
#define KB_NM(R) [](const ApplyArgs& a, hipStream_t s) { launch_lds<R, Policy<2, 1, true, true, false, 512, (R > 8 ? 4 : 2), 0, (R > 8 ? 1 : 0), true>>(a, s); }
        KB_NM(1), KB_NM(2), KB_NM(3), KB_NM(4), KB_NM(5), KB_NM(6), KB_NM(7), KB_NM(8),
        KB_NM(9), KB_NM(10), KB_NM(11), KB_NM(12), KB_NM(13), KB_NM(14), KB_NM(15), KB_NM(16)};
#undef KB_NM
    vs.push_back(Variant{"nomath g2 (ceiling)", [m](const ApplyArgs& a, hipStream_t s) { nomath_g2[m - 1](a, s); }, false});
    vs.push_back(Variant{"nomath consec (ceiling)", [m](const ApplyArgs& a, hipStream_t s) { nomath_c[m - 1](a, s); }, false});
  }
  if (rs10_4) vs.push_back(Variant{"read-only 10 streams (bytes: 10/14)", [](const ApplyArgs& a, hipStream_t s) {
                         const unsigned g = static_cast<unsigned>((a.nvec + 511) / 512 * a.batch);
                         hipLaunchKernelGGL((read_stream<10>), dim3(g), dim3(512), 0, s, a);
                       }, false});
  if (rs10_4) vs.push_back(Variant{"write-only 4 streams (bytes: 4/14)", [](const ApplyArgs& a, hipStream_t s) {
                         const unsigned g = static_cast<unsigned>((a.nvec + 511) / 512 * a.batch);
                         hipLaunchKernelGGL((write_stream<4>), dim3(g), dim3(512), 0, s, a);
                       }, false});
  if (rs10_4) vs.push_back(Variant{"xor-stream (ceiling)", [](const ApplyArgs& a, hipStream_t s) {
                         const unsigned g = static_cast<unsigned>((a.nvec + 255) / 256 * a.batch);
                         hipLaunchKernelGGL((xor_stream<10, 4, false>), dim3(g), dim3(256), 0, s, a);
                       }, false});
  if (rs10_4) vs.push_back(Variant{"xor-stream nt (ceiling)", [](const ApplyArgs& a, hipStream_t s) {
                         const unsigned g = static_cast<unsigned>((a.nvec + 255) / 256 * a.batch);
                         hipLaunchKernelGGL((xor_stream<10, 4, true>), dim3(g), dim3(256), 0, s, a);
                       }, false});
  vs.push_back(Variant{"hipMemcpy D2D same bytes/2", [&](const ApplyArgs&, hipStream_t s) {
                         // read+write of (k+m)/2*S per stripe: same total bytes moved
                         const size_t half = static_cast<size_t>(B) * n * pitch / 2;
                         CK(hipMemcpyAsync(buf + half, buf, half, hipMemcpyDeviceToDevice, s));
                       }, false});

  if (std::getenv("KB_PERSIST") && m <= 8) {  // persistent grids of N blocks per CU (small-S probe)
    // the production LDS policy (G8 order, ring of three) with PERSIST: a fixed grid of
    // 256 * N blocks strides over the tiles, so N bounds the tiles (and stripes) in flight
#define KB_PP Policy<2, 1, true, true, true, 512, 2, 2>
#define KB_PV(R) [](const ApplyArgs& a, hipStream_t s, unsigned g) { \
    hipLaunchKernelGGL((dev::rs_apply_lds<R, KB_PP>), dim3(g), dim3(512), dev::lds_bytes(a.K, R), s, a); }
    static void (*const pl[8])(const ApplyArgs&, hipStream_t, unsigned) = {
        KB_PV(1), KB_PV(2), KB_PV(3), KB_PV(4), KB_PV(5), KB_PV(6), KB_PV(7), KB_PV(8)};
#undef KB_PV
    static const int mm = m;
    for (int nb : {1, 2, 3, 4}) {
      static std::string names[5];
      names[nb] = "persist " + std::to_string(nb);
      vs.push_back(Variant{names[nb], [nb](const ApplyArgs& a, hipStream_t s) {
                             pl[mm - 1](a, s, dev::vec_grid<KB_PP>(a.nvec, a.batch, nb));
                           }});
    }
#undef KB_PP
  }
  // KB_ONLY=name: time only the variant of exactly that name (PMC passes of one variant)
  if (const char* only = std::getenv("KB_ONLY")) {
    std::vector<Variant> one;
    for (auto& v : vs)
      if (v.name == only) one.push_back(v);
    if (one.empty()) {
      std::fprintf(stderr, "KB_ONLY: no variant named %s\n", only);
      return 2;
    }
    vs.swap(one);
  }
  // KB_KEEP="a|b|...": keep only the variants whose name contains one of these (the
  // first variant, the production dispatch, is always kept: it is the parity reference)
  if (const char* keep = std::getenv("KB_KEEP")) {
    std::vector<std::string> pats;
    std::string ks(keep);
    for (size_t p = 0; p <= ks.size();) {
      size_t q = ks.find('|', p);
      if (q == std::string::npos) q = ks.size();
      if (q > p) pats.push_back(ks.substr(p, q - p));
      p = q + 1;
    }
    std::vector<Variant> kept{vs[0]};
    for (size_t i = 1; i < vs.size(); ++i)
      for (auto& pt : pats)
        if (vs[i].name.find(pt) != std::string::npos) {
          kept.push_back(vs[i]);
          break;
        }
    vs.swap(kept);
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // production reference parity
  vs[0].launch(a, s);
  CK(hipStreamSynchronize(s));
  CK(hipGetLastError());
  for (int b = 0; b < B; ++b)
    CK(hipMemcpy(ref + static_cast<size_t>(b) * m * opitch, out[b * m], m * opitch, hipMemcpyDeviceToDevice));

  // KB_VERIFY=mask: rows with these bits compare against the parity just written
  // (upstream Verify) instead of storing; the status word must stay 0
  const unsigned vmask = std::getenv("KB_VERIFY") ? std::strtoul(std::getenv("KB_VERIFY"), nullptr, 0) : 0;
  a.verify_mask = vmask;
  const double bytes = static_cast<double>(B) * S * n;
  std::vector<std::vector<double>> ms(vs.size());
  std::vector<uint8_t> h1(m * opitch), h2(m * opitch);
  for (int rd = 0; rd < rounds; ++rd) {
    // rotate the order each round: the variant timed right after the D2D copy ran
    // ~3 % slow when it always went first
    for (size_t vj = 0; vj < vs.size(); ++vj) {
      const size_t vi = (vj + rd) % vs.size();
      // warm for >= 30 ms, not a fixed count: the variant timed right after a no-lookup
      // ceiling kernel (light on VALU and LDS) ran 1.5-3 points slow on every shape
      // even after 4 warm launches (profiles/r02/prod_gap/, tail_check/) -- the clock
      // and power state of a light kernel carry over into the next one for milliseconds
      {
        float warm_ms = 0;
        for (int w = 0; w < 400 && warm_ms < 30.0f; w += 2) {
          CK(hipEventRecord(e0, s));
          vs[vi].launch(a, s);
          vs[vi].launch(a, s);
          CK(hipEventRecord(e1, s));
          CK(hipEventSynchronize(e1));
          float t = 0;
          CK(hipEventElapsedTime(&t, e0, e1));
          warm_ms += t;
        }
      }
      CK(hipEventRecord(e0, s));
      for (int it = 0; it < iters; ++it) vs[vi].launch(a, s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      CK(hipGetLastError());
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[vi].push_back(t / iters);
      if (rd == 0 && vs[vi].check) {
        for (int b : {0, B / 2, B - 1}) {
          CK(hipMemcpy(h1.data(), ref + static_cast<size_t>(b) * m * opitch, m * opitch, hipMemcpyDeviceToHost));
          CK(hipMemcpy(h2.data(), out[b * m], m * opitch, hipMemcpyDeviceToHost));
          bool same = true;
          for (int r = 0; r < m; ++r) same &= !std::memcmp(&h1[r * opitch], &h2[r * opitch], S);
          if (!same) std::printf("MISMATCH variant %s stripe %d\n", vs[vi].name.c_str(), b);
        }
      }
      // restore parity clobbered by ceiling kernels: needed for the round-0 parity checks
      // and for Verify runs (timing does not depend on the parity's contents)
      if (!vs[vi].check && vs[vi].name.rfind("probe", 0) != 0 && (rd == 0 || vmask)) {
        for (int b = 0; b < B; ++b)
          CK(hipMemcpy(out[b * m], ref + static_cast<size_t>(b) * m * opitch, m * opitch, hipMemcpyDeviceToDevice));
      }
    }
  }
  std::printf("RS(%d,%d) S=%zu pitch=%zu stripes=%d  working set %.2f GiB  rounds=%d iters=%d  in=%s out=%s\n",
              k, m, S, pitch, B, total / 1073741824.0, rounds, iters,
              std::getenv("KB_IN") ? std::getenv("KB_IN") : "0..k-1",
              std::getenv("KB_OUT") ? std::getenv("KB_OUT") : "k..n-1");
  if (vmask) {
    int st = 0;
    CK(hipMemcpy(&st, d_status, 4, hipMemcpyDeviceToHost));
    std::printf("verify_mask=0x%x status=%d%s\n", vmask, st, st ? "  MISMATCH (verify flagged)" : "");
  }
  std::printf("%-28s %10s %10s %10s %8s\n", "variant", "med_us", "min_us", "GB/s(med)", "%8TB/s");
  for (size_t vi = 0; vi < vs.size(); ++vi) {
    auto v = ms[vi];
    std::sort(v.begin(), v.end());
    const double med = v[v.size() / 2], mn = v[0];
    double frac = 1.0;
    if (vs[vi].name.rfind("read-only", 0) == 0) frac = static_cast<double>(k) / n;
    if (vs[vi].name.rfind("write-only", 0) == 0) frac = static_cast<double>(m) / n;
    if (vs[vi].name.find("bytes:") == std::string::npos && frac != 1.0)
      vs[vi].name += frac < 0.5 ? " (4/14)" : " (10/14)";
    const double gbs = bytes * frac / (med * 1e-3) / 1e9;
    std::printf("%-28s %10.1f %10.1f %10.1f %8.1f\n", vs[vi].name.c_str(), med * 1e3, mn * 1e3, gbs,
                gbs / 80.0);
  }
  return 0;
}
