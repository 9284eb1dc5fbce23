// ASan / UBSan driver for the HDF replay reader (madigan_amd/csrc/mgn_hdf.cpp,
// product host code; TEST INFRASTRUCTURE ONLY).  Built by `make -C oracle
// sanitize`, run by tests/test_sanitizers.py on the CPU (no GPU: every entry
// point but mgn_hdf_stage, whose H2D copies need a device).  Cases: the
// envTest.cpp:322-368 fixture and its bounds known answers, a multi-asset
// file, row reads at the edges, the cache-walk tape for several cache sizes,
// and the error paths (missing keys, out-of-range bounds, bad rows).
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../include/madigan_hdf.h"

static int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                     \
    }                                                              \
  } while (0)

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  // envTest.cpp:322-351: 10 rows, price i, feats i^3, timestamps i^2, asset "Test"
  const std::string kat = dir + "/sanitize_kat.h5";
  {
    std::vector<double> price(10), feats(10);
    std::vector<uint64_t> ts(10);
    for (int i = 0; i < 10; ++i) {
      price[i] = i;
      feats[i] = (double)i * i * i;
      ts[i] = (uint64_t)i * i;
    }
    const char* assets[] = {"Test"};
    CHECK(mgn_hdf_write(kat.c_str(), "group/dataset", "midprice", "feats", "timestamp", assets, 1, 10, 1,
                        price.data(), feats.data(), ts.data(), 1) == 0);
  }
  mgn_hdf* h = nullptr;
  CHECK(mgn_hdf_open(kat.c_str(), "group/dataset", "midprice", "feats", "timestamp", 0, 0, &h) == 0);
  mgn_hdf_info info{};
  CHECK(h && mgn_hdf_get_info(h, &info) == 0);
  CHECK(info.n_rows == 10 && info.first == 0 && info.second == 9 && info.end_time == 81);
  char code[8];
  CHECK(mgn_hdf_asset(h, 0, code, sizeof code) == 0 && std::string(code) == "Test");
  CHECK(mgn_hdf_asset(h, 0, code, 3) == 0);  // truncated
  CHECK(mgn_hdf_asset(h, 1, code, sizeof code) != 0);
  for (int64_t cs : {1, 3, 4, 10, 100}) {
    const int64_t n = mgn_hdf_tape_rows(h, cs);
    CHECK(n > 0);
    std::vector<int64_t> rows((size_t)n);
    CHECK(mgn_hdf_tape_index(h, cs, rows.data()) == 0);
    for (int64_t r : rows) CHECK(r >= 0 && r < 10);
  }
  {
    std::vector<double> p(10), f(10);
    std::vector<uint64_t> t(10);
    CHECK(mgn_hdf_read(h, 0, 10, p.data(), f.data(), t.data()) == 0 && p[9] == 9.0 && f[2] == 8.0);
    CHECK(mgn_hdf_read(h, 9, 1, p.data(), nullptr, t.data()) == 0);
    CHECK(mgn_hdf_read(h, 5, 10, p.data(), f.data(), t.data()) != 0);
    CHECK(mgn_hdf_read(h, -1, 2, p.data(), f.data(), t.data()) != 0);
  }
  CHECK(mgn_hdf_close(h) == 0);
  // envTest.cpp:386-397: bounds for [1, 63] are (1, 7); [0, 82] throws out_of_range
  CHECK(mgn_hdf_open(kat.c_str(), "group/dataset", "midprice", "feats", "timestamp", 1, 63, &h) == 0);
  CHECK(mgn_hdf_get_info(h, &info) == 0 && info.first == 1 && info.second == 7);
  CHECK(mgn_hdf_close(h) == 0);
  h = nullptr;
  CHECK(mgn_hdf_open(kat.c_str(), "group/dataset", "midprice", "feats", "timestamp", 0, 82, &h) != 0);
  CHECK(mgn_hdf_open(kat.c_str(), "group/dataset", "nope", "feats", "timestamp", 0, 0, &h) != 0);
  CHECK(mgn_hdf_open(kat.c_str(), "group/other", "midprice", "feats", "timestamp", 0, 0, &h) != 0);
  CHECK(mgn_hdf_open((dir + "/missing.h5").c_str(), "g", "p", "f", "t", 0, 0, &h) != 0);
  CHECK(mgn_hdf_last_error() != nullptr);
  // multi-asset (T, A) layout with ragged cache sizes
  const std::string multi = dir + "/sanitize_multi.h5";
  {
    const int T = 37, A = 3, F = 5;
    std::vector<double> price(T * A), feats(T * F);
    std::vector<uint64_t> ts(T);
    for (int t = 0; t < T; ++t) {
      ts[t] = 100 + 7 * (uint64_t)t;
      for (int a = 0; a < A; ++a) price[t * A + a] = 10.0 + t + 0.1 * a;
      for (int j = 0; j < F; ++j) feats[t * F + j] = t - j;
    }
    const char* assets[] = {"A", "BB", "CCC"};
    CHECK(mgn_hdf_write(multi.c_str(), "fx/daily", "price", "features", "timestamps", assets, A, T, F,
                        price.data(), feats.data(), ts.data(), 0) == 0);
    CHECK(mgn_hdf_open(multi.c_str(), "fx/daily", "price", "features", "timestamps", 120, 300, &h) == 0);
    CHECK(mgn_hdf_get_info(h, &info) == 0 && info.n_assets == A && info.n_feats == F && !info.price_1d);
    for (int64_t cs : {1, 2, 5, 7, 1000}) {
      const int64_t n = mgn_hdf_tape_rows(h, cs);
      std::vector<int64_t> rows((size_t)(n > 0 ? n : 1));
      CHECK(n > 0 && mgn_hdf_tape_index(h, cs, rows.data()) == 0);
    }
    std::vector<double> p(4 * A), f(4 * F);
    std::vector<uint64_t> t(4);
    CHECK(mgn_hdf_read(h, 33, 4, p.data(), f.data(), t.data()) == 0 && p[3 * A + 2] == 10.0 + 36 + 0.2);
    CHECK(mgn_hdf_close(h) == 0);
  }
  std::remove(kat.c_str());
  std::remove(multi.c_str());
  if (fails) return 1;
  std::printf("sanitize_hdf: all cases clean\n");
  return 0;
}
