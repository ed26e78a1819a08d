// Host-side GF(2^8) arithmetic and coding matrices for the RS path.
//
// Field and matrix construction match github.com/klauspost/reedsolomon v1.13.3
// (go.mod:13), reached from erasure/codec.go:26,50 via reedsolomon.New:
//   field   GF(2^8) mod x^8+x^4+x^3+x^2+1 (0x11D), generator 2
//   matrix  E = V . inv(V[0:k]), V[r][c] = r^c with 0^0 = 1   (systematic; E[0:k] = I)
//   decode  first k present shards (index order), D = inv(E[valid])  (codec.go:55)
// Everything here is O(n*k^2) host work on at most 256x256 bytes; the byte streams
// are processed by the HIP kernels in rs_kernels.hip.
#pragma once

#include <array>
#include <cstdint>
#include <cstring>
#include <vector>

namespace callfs {

struct GF {
  std::array<uint8_t, 512> exp{};
  std::array<uint8_t, 256> log{};
  std::array<std::array<uint8_t, 256>, 256> mul{};

  GF() {
    unsigned x = 1;
    for (int i = 0; i < 255; ++i) {
      exp[i] = static_cast<uint8_t>(x);
      log[x] = static_cast<uint8_t>(i);
      x <<= 1;
      if (x & 0x100u) x ^= 0x11Du;
    }
    for (int i = 255; i < 512; ++i) exp[i] = exp[i - 255];
    for (int a = 0; a < 256; ++a)
      for (int b = 0; b < 256; ++b)
        mul[a][b] = (a && b) ? exp[log[a] + log[b]] : 0;
  }
  uint8_t inv(uint8_t a) const { return exp[(255 - log[a]) % 255]; }
  uint8_t pow(uint8_t a, int n) const {
    if (n == 0) return 1;
    if (a == 0) return 0;
    return exp[(static_cast<int>(log[a]) * n) % 255];
  }
};

inline const GF& gf() {
  static const GF g;
  return g;
}

// Row-major byte matrix.
struct Mat {
  int rows = 0, cols = 0;
  std::vector<uint8_t> v;
  Mat() = default;
  Mat(int r, int c) : rows(r), cols(c), v(static_cast<size_t>(r) * c, 0) {}
  uint8_t& at(int r, int c) { return v[static_cast<size_t>(r) * cols + c]; }
  uint8_t at(int r, int c) const { return v[static_cast<size_t>(r) * cols + c]; }
  const uint8_t* row(int r) const { return v.data() + static_cast<size_t>(r) * cols; }
};

inline Mat matmul(const Mat& a, const Mat& b) {
  const GF& g = gf();
  Mat o(a.rows, b.cols);
  for (int r = 0; r < a.rows; ++r)
    for (int i = 0; i < a.cols; ++i) {
      uint8_t x = a.at(r, i);
      if (!x) continue;
      const uint8_t* mt = g.mul[x].data();
      for (int c = 0; c < b.cols; ++c) o.at(r, c) ^= mt[b.at(i, c)];
    }
  return o;
}

// Gauss-Jordan inversion; false when singular.
inline bool invert(const Mat& in, Mat& out) {
  const GF& g = gf();
  const int n = in.rows;
  Mat w(n, 2 * n);
  for (int r = 0; r < n; ++r) {
    std::memcpy(&w.at(r, 0), in.row(r), n);
    w.at(r, n + r) = 1;
  }
  for (int r = 0; r < n; ++r) {
    if (w.at(r, r) == 0) {
      for (int b = r + 1; b < n; ++b)
        if (w.at(b, r)) {
          for (int c = 0; c < 2 * n; ++c) std::swap(w.at(r, c), w.at(b, c));
          break;
        }
    }
    if (w.at(r, r) == 0) return false;
    const uint8_t s = g.inv(w.at(r, r));
    for (int c = 0; c < 2 * n; ++c) w.at(r, c) = g.mul[s][w.at(r, c)];
    for (int o = 0; o < n; ++o) {
      if (o == r || !w.at(o, r)) continue;
      const uint8_t* mt = g.mul[w.at(o, r)].data();
      for (int c = 0; c < 2 * n; ++c) w.at(o, c) ^= mt[w.at(r, c)];
    }
  }
  out = Mat(n, n);
  for (int r = 0; r < n; ++r) std::memcpy(&out.at(r, 0), &w.at(r, n), n);
  return true;
}

// Systematic encoding matrix E ((k+m) x k).
inline bool encode_matrix(int k, int m, Mat& E) {
  const GF& g = gf();
  const int n = k + m;
  Mat V(n, k);
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < k; ++c) V.at(r, c) = g.pow(static_cast<uint8_t>(r), c);
  Mat top(k, k), ti;
  for (int r = 0; r < k; ++r) std::memcpy(&top.at(r, 0), V.row(r), k);
  if (!invert(top, ti)) return false;
  E = matmul(V, ti);
  return true;
}

// Rows over the first k present shards that produce each missing shard, and the
// present parity shards beyond the first k (those Verify must re-check).
struct DecodePlan {
  std::vector<int> valid;    // k shard indices read
  std::vector<int> missing;  // shard indices written
  std::vector<int> check;    // present parity indices compared (Verify)
  Mat rows;                  // (missing + check) x k; missing rows first
};

// present: n flags. Returns false when singular (cannot happen for k+m <= 256).
inline bool decode_plan(int k, int m, const uint8_t* present, DecodePlan& p) {
  const int n = k + m;
  Mat E;
  if (!encode_matrix(k, m, E)) return false;
  p.valid.clear(); p.missing.clear(); p.check.clear();
  for (int i = 0; i < n; ++i) {
    if (present[i]) {
      if (static_cast<int>(p.valid.size()) < k) p.valid.push_back(i);
      else p.check.push_back(i);  // always a parity index: data indices come first
    } else {
      p.missing.push_back(i);
    }
  }
  Mat sub(k, k), D;
  for (int r = 0; r < k; ++r) std::memcpy(&sub.at(r, 0), E.row(p.valid[r]), k);
  if (!invert(sub, D)) return false;
  const int R = static_cast<int>(p.missing.size() + p.check.size());
  p.rows = Mat(R, k);
  int r = 0;
  auto emit = [&](int idx) {
    if (idx < k) {
      std::memcpy(&p.rows.at(r, 0), D.row(idx), k);
    } else {
      Mat er(1, k);
      std::memcpy(&er.at(0, 0), E.row(idx), k);
      Mat pr = matmul(er, D);
      std::memcpy(&p.rows.at(r, 0), pr.row(0), k);
    }
    ++r;
  };
  for (int idx : p.missing) emit(idx);
  for (int idx : p.check) emit(idx);
  return true;
}

// v_perm_b32 lookup tables for multiplying 4 packed bytes by coefficient c:
//   c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6]
// T0/T1 are 8-byte tables (lo dword = entries 0..3, hi dword = entries 4..7, the
// {S0=hi, S1=lo} byte order of v_perm_b32); T2 has 4 entries in one dword.
constexpr int kTabWords = 5;
inline void perm_tables(uint8_t c, uint32_t out[kTabWords]) {
  const GF& g = gf();
  uint8_t t0[8], t1[8], t2[4];
  for (int x = 0; x < 8; ++x) {
    t0[x] = g.mul[c][x];
    t1[x] = g.mul[c][x << 3];
  }
  for (int x = 0; x < 4; ++x) t2[x] = g.mul[c][x << 6];
  auto pack = [](const uint8_t* b) {
    return static_cast<uint32_t>(b[0]) | (static_cast<uint32_t>(b[1]) << 8) |
           (static_cast<uint32_t>(b[2]) << 16) | (static_cast<uint32_t>(b[3]) << 24);
  };
  out[0] = pack(t0);      // T0 lo
  out[1] = pack(t0 + 4);  // T0 hi
  out[2] = pack(t1);      // T1 lo
  out[3] = pack(t1 + 4);  // T1 hi
  out[4] = pack(t2);      // T2
}

// LDS nibble tables for one input shard over R output rows, entries of W bytes
// (W = 8 for R <= 8, 16 for R <= 16): entry e (0..15) of the low table holds c_r * e in
// byte r, entry e of the high table c_r * (e << 4); out = low[16][W] then high[16][W],
// 32*W bytes per shard. A 16-entry table of W-byte entries spans 16*W/4 distinct LDS
// banks (32 or all 64), so random lookups never conflict (rs_apply.hpp rs_apply_lds).
inline int nibble_width(int R) { return R > 8 ? 16 : 8; }

inline void nibble_tables(const uint8_t* coef_rows, int R, uint8_t* out) {
  const GF& g = gf();
  const int W = nibble_width(R);
  std::memset(out, 0, static_cast<size_t>(32) * W);
  for (int e = 0; e < 16; ++e)
    for (int r = 0; r < R && r < W; ++r) {
      out[e * W + r] = g.mul[coef_rows[r]][e];
      out[(16 + e) * W + r] = g.mul[coef_rows[r]][e << 4];
    }
}

}  // namespace callfs
