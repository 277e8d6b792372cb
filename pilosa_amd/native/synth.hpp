// Deterministic synthetic set-field generator (shared by the in-memory arena
// builder in pyroaring.cpp and the fragment-file writer in arena_io.cpp).
//
// Row r has column density d_r = min(1, bits_per_col * (v+r)^-s / Z),
// Z = sum_k (v+k)^-s, i.e. the reference's Zipf(s=1.6, v=50) row generator
// (fragment_internal_test.go:2377-2460) drawn bits_per_col times per column.
// Sparse row-shards draw Poisson(d_r * cols) uniform positions; dense ones draw
// a per-container count and place it stratified (distinct, sorted).  Every
// (seed, shard, row) triple has its own RNG stream, so a shard's contents do
// not depend on which process or thread generates it.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "roaring.hpp"

namespace synth {

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uni() { return double(next() >> 11) * (1.0 / 9007199254740992.0); }
  int64_t poisson(double lam) {
    if (lam <= 0) return 0;
    if (lam < 30) {
      double L = std::exp(-lam), p = 1.0;
      int64_t k = 0;
      do { k++; p *= uni(); } while (p > L);
      return k - 1;
    }
    double u1 = std::max(uni(), 1e-300), u2 = uni();
    double z = std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
    int64_t k = int64_t(std::llround(lam + std::sqrt(lam) * z));
    return k < 0 ? 0 : k;
  }
};

inline uint64_t mix3(uint64_t a, uint64_t b, uint64_t c) {
  Rng r(a * 0x100000001B3ull ^ (b << 21) ^ (c * 0xD6E8FEB86659FD93ull));
  r.next();
  return r.next();
}

// One shard in the device arena layout (rowptr relative, meta payload offsets
// relative to the shard; meta packing documented in pyroaring.cpp).
struct ShardOut {
  std::vector<uint32_t> rowptr;
  std::vector<int64_t> meta;
  std::vector<uint16_t> payload;
  // n values sorted distinct (vals) or bitmap words (w) when n > 4096
  void emit(int j, const uint16_t* vals, int n, const uint64_t* w) {
    const int64_t off = int64_t(payload.size());
    int type;
    if (n <= pr::ARRAY_MAX) {
      type = pr::CT_ARRAY;
      payload.insert(payload.end(), vals, vals + n);
      payload.resize((payload.size() + 7) & ~size_t(7), 0);
    } else {
      type = pr::CT_BITMAP;
      const uint16_t* p = reinterpret_cast<const uint16_t*>(w);
      payload.insert(payload.end(), p, p + 4096);
    }
    meta.push_back(int64_t(uint64_t(j) | (uint64_t(type) << 4) | (uint64_t(n) << 6) | (uint64_t(off / 8) << 23)));
  }
  // emit a container from bitmap words (array when sparse)
  void emit_words(int j, const uint64_t* w, std::vector<uint16_t>& tmp) {
    int n = 0;
    for (int i = 0; i < 1024; i++) n += __builtin_popcountll(w[i]);
    if (n == 0) return;
    if (n > pr::ARRAY_MAX) {
      emit(j, nullptr, n, w);
      return;
    }
    tmp.clear();
    for (int i = 0; i < 1024; i++)
      for (uint64_t b = w[i]; b; b &= b - 1) tmp.push_back(uint16_t(i * 64 + __builtin_ctzll(b)));
    emit(j, tmp.data(), n, nullptr);
  }
};

// Per-row column densities of the Zipf set field.
inline std::vector<double> zipf_densities(int64_t nrows, double bits_per_col, double zs, double zv) {
  std::vector<double> dens(size_t(std::max<int64_t>(nrows, 0)));
  double Z = 0;
  for (int64_t r = 0; r < nrows; r++) Z += std::pow(zv + double(r), -zs);
  for (int64_t r = 0; r < nrows; r++) dens[size_t(r)] = std::min(1.0, bits_per_col * std::pow(zv + double(r), -zs) / Z);
  return dens;
}

// Generate one shard of the Zipf set field (rows 0..R-1) into o.
inline void gen_zipf_shard(ShardOut& o, int64_t shard, int64_t total_cols, const std::vector<double>& dens,
                           uint64_t seed) {
  const int64_t R = int64_t(dens.size());
  const int64_t cols = std::max<int64_t>(0, std::min<int64_t>(1 << 20, total_cols - shard * (1 << 20)));
  std::vector<uint64_t> pos;
  std::vector<uint64_t> words(1024);
  std::vector<uint16_t> vals;
  o.rowptr.assign(size_t(R + 1), 0);
  for (int64_t r = 0; r < R; r++) {
    o.rowptr[size_t(r)] = uint32_t(o.meta.size());
    if (cols == 0) continue;
    Rng rng(mix3(seed, uint64_t(shard), uint64_t(r)));
    const double lam_row = dens[size_t(r)] * double(cols);
    if (lam_row < 2048.0) {
      int64_t N = rng.poisson(lam_row);
      if (N == 0) continue;
      pos.resize(size_t(N));
      for (int64_t k = 0; k < N; k++) pos[size_t(k)] = rng.next() % uint64_t(cols);
      std::sort(pos.begin(), pos.end());
      pos.erase(std::unique(pos.begin(), pos.end()), pos.end());
      size_t i = 0;
      while (i < pos.size()) {
        int j = int(pos[i] >> 16);
        vals.clear();
        while (i < pos.size() && int(pos[i] >> 16) == j) vals.push_back(uint16_t(pos[i] & 0xffff)), i++;
        o.emit(j, vals.data(), int(vals.size()), nullptr);
      }
    } else {
      for (int j = 0; j < 16; j++) {
        const int64_t lim = std::min<int64_t>(65536, cols - int64_t(j) * 65536);
        if (lim <= 0) break;
        int64_t n = dens[size_t(r)] >= 1.0 ? lim : rng.poisson(dens[size_t(r)] * double(lim));
        n = std::min<int64_t>(n, lim);
        if (n == 0) continue;
        // stratified distinct positions
        vals.resize(size_t(n));
        for (int64_t k = 0; k < n; k++) {
          int64_t a = k * lim / n, b = (k + 1) * lim / n;
          vals[size_t(k)] = uint16_t(a + int64_t(rng.next() % uint64_t(std::max<int64_t>(1, b - a))));
        }
        if (n > pr::ARRAY_MAX) {
          std::fill(words.begin(), words.end(), 0);
          for (int64_t k = 0; k < n; k++) words[vals[size_t(k)] >> 6] |= 1ull << (vals[size_t(k)] & 63);
          o.emit(j, nullptr, int(n), words.data());
        } else {
          o.emit(j, vals.data(), int(n), nullptr);
        }
      }
    }
  }
  o.rowptr[size_t(R)] = uint32_t(o.meta.size());
}

// One shard of a synthetic BSI int field (reference bsiExistsBit / bsiSignBit /
// bsiOffsetBit layout, sign-magnitude): a fraction `fill` of the columns hold
// a value uniform in [vmin, vmax]; rows 0 = exists, 1 = sign, 2+i = bit i of
// |value|.  Deterministic per (seed, shard).
inline void gen_bsi_shard(ShardOut& o, int64_t shard, int64_t total_cols, int depth, double fill, int64_t vmin,
                          int64_t vmax, uint64_t seed) {
  const int64_t cols = std::max<int64_t>(0, std::min<int64_t>(1 << 20, total_cols - shard * (1 << 20)));
  const int64_t R = depth + 2;
  o.rowptr.assign(size_t(R + 1), 0);
  std::vector<uint64_t> planes(size_t(R) * 16 * 1024, 0);  // planes[r][j][1024]
  Rng rng(mix3(seed, uint64_t(shard), 0xB51));
  const uint64_t span = uint64_t(vmax - vmin) + 1;
  for (int64_t c = 0; c < cols; c++) {
    if (double(rng.next() >> 11) * (1.0 / 9007199254740992.0) >= fill) continue;
    const int64_t v = vmin + int64_t(rng.next() % span);
    const uint64_t u = uint64_t(v < 0 ? -v : v);
    const int j = int(c >> 16), w = int((c & 0xffff) >> 6);
    const uint64_t bit = 1ull << (c & 63);
    planes[(size_t(0) * 16 + size_t(j)) * 1024 + size_t(w)] |= bit;
    if (v < 0) planes[(size_t(1) * 16 + size_t(j)) * 1024 + size_t(w)] |= bit;
    for (int i = 0; i < depth; i++)
      if ((u >> i) & 1) planes[(size_t(2 + i) * 16 + size_t(j)) * 1024 + size_t(w)] |= bit;
  }
  std::vector<uint16_t> tmp;
  for (int64_t r = 0; r < R; r++) {
    o.rowptr[size_t(r)] = uint32_t(o.meta.size());
    for (int j = 0; j < 16; j++) o.emit_words(j, &planes[(size_t(r) * 16 + size_t(j)) * 1024], tmp);
  }
  o.rowptr[size_t(R)] = uint32_t(o.meta.size());
}

}  // namespace synth
