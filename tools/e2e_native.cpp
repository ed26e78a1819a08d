// End-to-end host-memory RS throughput through the C ABI from native threads — the way
// the Go server's request goroutines would call it (one cgo call per request), without
// Python in the loop. Development tool, not product.
//
// build: g++ -O2 -std=c++17 -I include tools/e2e_native.cpp -L callfs_amd -lcallfs_rs \
//          -Wl,-rpath,'$ORIGIN/../callfs_amd' -lpthread -o tools/e2e_native
// run:   tools/e2e_native k m object_bytes threads seconds [erase,list]
// CALLFS_E2E_ENCODER=1: encode through rs_encode (Go-side Split aliasing the object,
// parity only, as INTEGRATION.md's shim does) instead of rs_codec_encode.
// CALLFS_E2E_BATCH=N: each call handles N objects through rs_encode_batch /
// rs_reconstruct_batch (verify on) plus the per-object join copy.
// CALLFS_E2E_PINNED=1: every buffer comes from rs_host_alloc (the server reading bodies
// and shards into pinned memory), so calls take the zero-copy direct-DMA path.
// Zero-copy concurrency probes:
// CALLFS_E2E_EXTRA_PINNED_MIB=N: also hold N MiB of touched, unused rs_host_alloc memory
//   (a larger pinned footprint without more concurrent calls);
// CALLFS_E2E_SERIAL=1: one rs_* call at a time across all threads (concurrency without
//   overlap: same footprint, calls serialised by a mutex in this harness);
// CALLFS_E2E_FRESH=1: allocate (and free) the output buffers of every call anew.
// CALLFS_E2E_BODY=1: the shim's pinned-body path exactly as tests/native/cgo_drive.c drives
//   it (codec_rocm.go BodyBuffer -> Encode, DecodePinned, FreeHostBuffer): each encode takes a
//   body of n*S bytes from rs_host_alloc (the context's pool after the first call), holding
//   the object in its first L bytes as io.ReadFull left it, zeroes the spare capacity as Split
//   does, encodes in place with rs_encode and frees the body; each decode allocates the lost
//   shards' and the object's buffers from rs_host_alloc, runs rs_codec_decode and frees them
//   (the fetched shards are pinned buffers filled once).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <random>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "callfs_rs.h"

// Allocator for every buffer of the run: rs_host_alloc memory when CALLFS_E2E_PINNED is
// set, plain heap otherwise.
static rs_ctx* g_ctx = nullptr;
static bool g_pinned = false;
template <class T>
struct MaybePinned {
  using value_type = T;
  MaybePinned() = default;
  template <class U>
  MaybePinned(const MaybePinned<U>&) {}
  T* allocate(size_t n) {
    if (!g_pinned) return static_cast<T*>(::operator new(n * sizeof(T)));
    void* p = nullptr;
    if (rs_host_alloc(g_ctx, std::max<size_t>(1, n * sizeof(T)), &p) != RS_OK) throw std::bad_alloc();
    return static_cast<T*>(p);
  }
  void deallocate(T* p, size_t) {
    if (!g_pinned) ::operator delete(p);
    else rs_host_free(g_ctx, p);
  }
  // default-initialise (no zero fill): a fresh per-call buffer costs what the server's
  // allocation would, not a memset of the whole object
  template <class U>
  void construct(U* p) { ::new (static_cast<void*>(p)) U; }
  template <class U, class... A>
  void construct(U* p, A&&... a) { ::new (static_cast<void*>(p)) U(std::forward<A>(a)...); }
  template <class U>
  bool operator==(const MaybePinned<U>&) const { return true; }
  template <class U>
  bool operator!=(const MaybePinned<U>&) const { return false; }
};
using Bytes = std::vector<uint8_t, MaybePinned<uint8_t>>;

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s k m object_bytes threads seconds [erase,list]\n", argv[0]);
    return 2;
  }
  const int k = std::atoi(argv[1]), m = std::atoi(argv[2]), n = k + m;
  const size_t L = std::strtoull(argv[3], nullptr, 0);
  const int T = std::atoi(argv[4]);
  const double secs = std::atof(argv[5]);
  std::vector<int> erase;
  if (argc > 6) {
    std::string e(argv[6]);
    for (size_t p = 0; p < e.size();) {
      size_t q = e.find(',', p);
      if (q == std::string::npos) q = e.size();
      if (q > p) erase.push_back(std::atoi(e.substr(p, q - p).c_str()));
      p = q + 1;
    }
  }
  const bool encoder_api = std::getenv("CALLFS_E2E_ENCODER") != nullptr;
  const bool body_api = std::getenv("CALLFS_E2E_BODY") != nullptr;
  const int nb = std::getenv("CALLFS_E2E_BATCH") ? std::atoi(std::getenv("CALLFS_E2E_BATCH")) : 0;
  rs_ctx* ctx = nullptr;
  if (rs_init(&ctx, 0) != RS_OK) {
    std::fprintf(stderr, "rs_init failed\n");
    return 1;
  }
  g_ctx = ctx;
  g_pinned = std::getenv("CALLFS_E2E_PINNED") != nullptr || body_api;
  const size_t S = (L + k - 1) / k;
  const bool serial = std::getenv("CALLFS_E2E_SERIAL") != nullptr;
  const bool fresh = std::getenv("CALLFS_E2E_FRESH") != nullptr;
  static std::mutex call_mu;
  std::vector<void*> extra;  // 1 GiB pieces (one huge pinned allocation can fail)
  if (const char* x = std::getenv("CALLFS_E2E_EXTRA_PINNED_MIB")) {
    for (size_t left = std::strtoull(x, nullptr, 0) << 20; left;) {
      const size_t piece = std::min<size_t>(left, 1ull << 30);
      void* p = nullptr;
      if (rs_host_alloc(ctx, piece, &p) != RS_OK) {
        std::fprintf(stderr, "rs_host_alloc(%zu) failed\n", piece);
        return 1;
      }
      for (size_t i = 0; i < piece; i += 4096) static_cast<uint8_t*>(p)[i] = static_cast<uint8_t>(i >> 12);
      extra.push_back(p);
      left -= piece;
    }
  }
  struct Thr {
    Bytes src, enc, out;
    std::vector<Bytes> sh;
    long ops = 0;
    int err = 0;
  };
  auto th_holder = std::make_unique<std::vector<Thr>>(T);
  std::vector<Thr>& th = *th_holder;
  for (int t = 0; t < T; ++t) {
    std::mt19937_64 rng(1234 + t);
    th[t].src.resize(L);
    for (auto& b : th[t].src) b = static_cast<uint8_t>(rng());
    th[t].enc.resize(n * S);
    th[t].out.resize(L);
    size_t ss = 0;
    if (rs_codec_encode(ctx, k, m, th[t].src.data(), L, th[t].enc.data(), n * S, &ss) != RS_OK) return 1;
    th[t].sh.assign(n, Bytes(S));
    for (int i = 0; i < n; ++i) std::memcpy(th[t].sh[i].data(), th[t].enc.data() + S * i, S);
  }
  auto run = [&](bool encode) {
    std::atomic<bool> stop{false};
    std::vector<std::thread> ws;
    for (int t = 0; t < T; ++t) {
      th[t].ops = 0;
      ws.emplace_back([&, t] {
        Thr& me = th[t];
        Bytes enc2(n * S);
        std::vector<uint8_t*> ptrs(n);
        std::vector<size_t> lens(n);
        // batch mode: every object shares the same input bytes, outputs are per object
        const int B = nb > 0 ? nb : 1;
        Bytes bout(nb > 0 ? static_cast<size_t>(B) * n * S : 0);
        std::vector<const uint8_t*> bdata(nb > 0 ? static_cast<size_t>(B) * k : 0);
        std::vector<uint8_t*> bpar(nb > 0 ? static_cast<size_t>(B) * m : 0);
        std::vector<uint8_t*> bsh(nb > 0 ? static_cast<size_t>(B) * n : 0);
        std::vector<size_t> bsz(B, S), blens(nb > 0 ? static_cast<size_t>(B) * n : 0);
        std::vector<int> bst(B);
        Bytes bjoin(nb > 0 ? L : 0);
        while (!stop.load(std::memory_order_relaxed)) {
          int rc;
          std::unique_lock<std::mutex> serial_lock(call_mu, std::defer_lock);
          if (serial) serial_lock.lock();
          if (fresh) Bytes(n * S).swap(enc2);  // new pinned output buffer for this call
          if (nb > 0 && encode) {
            for (int b = 0; b < B; ++b) {
              for (int i = 0; i < k; ++i) bdata[static_cast<size_t>(b) * k + i] = me.enc.data() + S * i;
              for (int j = 0; j < m; ++j)
                bpar[static_cast<size_t>(b) * m + j] = bout.data() + (static_cast<size_t>(b) * n + k + j) * S;
            }
            rc = rs_encode_batch(ctx, k, m, B, bsz.data(), bdata.data(), bpar.data(), bst.data());
          } else if (nb > 0) {
            for (int b = 0; b < B; ++b)
              for (int i = 0; i < n; ++i) {
                bool gone = false;
                for (int e : erase) gone |= e == i;
                const size_t x = static_cast<size_t>(b) * n + i;
                bsh[x] = gone ? bout.data() + x * S : me.sh[i].data();
                blens[x] = gone ? 0 : S;
              }
            rc = rs_reconstruct_batch(ctx, k, m, B, bsh.data(), blens.data(), 1, bst.data());
            for (int b = 0; b < B && rc == RS_OK; ++b) {  // join + trim per object
              size_t left = L;
              for (int i = 0; i < k && left; ++i) {
                const size_t c = std::min(S, left);
                std::memcpy(bjoin.data() + S * i, bsh[static_cast<size_t>(b) * n + i], c);
                left -= c;
              }
              if (b == 0) me.out = bjoin;
            }
          } else if (encode && body_api) {
            uint8_t* body = nullptr;
            rc = rs_host_alloc(ctx, n * S, reinterpret_cast<void**>(&body));
            if (rc == RS_OK) {
              // the body as io.ReadFull leaves it: the object's L bytes (written once per
              // thread into the first body; a pool body holds the last request's object)
              if (me.ops == 0) std::memcpy(body, me.src.data(), L);
              std::memset(body + L, 0, n * S - L);  // Split zeroes the spare capacity
              std::vector<const uint8_t*> dptr(k);
              std::vector<uint8_t*> pptr(m);
              for (int i = 0; i < k; ++i) dptr[i] = body + S * i;
              for (int j = 0; j < m; ++j) pptr[j] = body + S * (k + j);
              rc = rs_encode(ctx, k, m, S, dptr.data(), pptr.data());
              if (rs_host_free(ctx, body) != RS_OK && rc == RS_OK) rc = RS_E_ARG;
            }
          } else if (!encode && body_api) {
            // DecodePinned: the lost entries and the object come from rs_host_alloc per call
            std::vector<void*> mine;
            rc = RS_OK;
            for (int i = 0; i < n && rc == RS_OK; ++i) {
              bool gone = false;
              for (int e : erase) gone |= e == i;
              lens[i] = gone ? 0 : S;
              ptrs[i] = me.sh[i].data();
              if (gone) {
                void* b = nullptr;
                rc = rs_host_alloc(ctx, S, &b);
                ptrs[i] = static_cast<uint8_t*>(b);
                mine.push_back(b);
              }
            }
            void* ob = nullptr;
            if (rc == RS_OK) rc = rs_host_alloc(ctx, L, &ob);
            if (rc == RS_OK)
              rc = rs_codec_decode(ctx, k, m, ptrs.data(), lens.data(), static_cast<uint8_t*>(ob),
                                   static_cast<int64_t>(L));
            if (rc == RS_OK && me.ops == 0) std::memcpy(me.out.data(), ob, L);
            if (ob) mine.push_back(ob);
            for (void* b : mine) rs_host_free(ctx, b);
          } else if (encode && encoder_api) {
            // Split as upstream: full data shards alias src, the tail shard is a
            // zero-padded copy, parity lands in fresh buffers
            const size_t full = L / S;
            std::vector<const uint8_t*> dptr(k);
            std::vector<uint8_t*> pptr(m);
            for (size_t i = 0; i < full; ++i) dptr[i] = me.src.data() + S * i;
            for (int i = static_cast<int>(full); i < k; ++i) {
              uint8_t* t = enc2.data() + S * i;
              const size_t have = i == static_cast<int>(full) ? L - full * S : 0;
              std::memcpy(t, me.src.data() + full * S, have);
              std::memset(t + have, 0, S - have);
              dptr[i] = t;
            }
            for (int j = 0; j < m; ++j) pptr[j] = enc2.data() + S * (k + j);
            rc = rs_encode(ctx, k, m, S, dptr.data(), pptr.data());
          } else if (encode) {
            size_t ss = 0;
            rc = rs_codec_encode(ctx, k, m, me.src.data(), L, enc2.data(), n * S, &ss);
          } else {
            // present shards were fetched once before the loop; the erased ones are
            // rebuilt into their buffers by every call
            for (int i = 0; i < n; ++i) {
              bool gone = false;
              for (int e : erase) gone |= e == i;
              ptrs[i] = me.sh[i].data();
              lens[i] = gone ? 0 : S;
            }
            rc = rs_codec_decode(ctx, k, m, ptrs.data(), lens.data(), me.out.data(),
                                 static_cast<int64_t>(L));
          }
          if (rc != RS_OK) me.err = rc;
          me.ops += B;
        }
      });
    }
    const auto t0 = std::chrono::steady_clock::now();
    std::this_thread::sleep_for(std::chrono::duration<double>(secs));
    stop = true;
    for (auto& w : ws) w.join();
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    long ops = 0;
    for (auto& x : th) ops += x.ops;
    return std::make_pair(ops / el * L / 1073741824.0, ops);
  };
  auto e = run(true);
  auto d = run(false);
  int bad = 0;
  for (auto& x : th) bad |= x.err || x.out != x.src;
  std::printf("{\"api\": \"%s\", \"k\": %d, \"m\": %d, \"object_bytes\": %zu, \"threads\": %d, "
              "\"batch\": %d, \"erase_count\": %zu, \"encode_gib_s\": %.3f, \"decode_gib_s\": %.3f, "
              "\"encode_calls\": %ld, \"decode_calls\": %ld, \"ok\": %s}\n",
              nb > 0 ? (g_pinned ? "native-batch-pinned" : "native-batch")
                     : body_api ? "native-body-pinned"
                     : encoder_api ? (g_pinned ? "native-encoder-pinned" : "native-encoder")
                                   : (g_pinned ? "native-pinned" : "native"),
              k, m, L, T, nb > 0 ? nb : 1, erase.size(), e.first, d.first, e.second, d.second,
              bad ? "false" : "true");
  th_holder.reset();  // pinned buffers go back before the context
  for (void* p : extra) rs_host_free(ctx, p);
  rs_shutdown(ctx);
  return bad ? 1 : 0;
}
