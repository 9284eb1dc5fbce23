// mgn_hdf.cpp -- HDF replay DataSource for the MI355X path (include/madigan_hdf.h).
//
// Host code: libhdf5's C API for the file, the HIP runtime for pinned staging
// buffers and asynchronous H2D copies.  The replay "tape" is one period of the
// row sequence HDFSourceSingle::getData visits (iterCache / loadData,
// DataSource.cpp:368-408): a concatenation of contiguous chunks, one per cache
// refill, which mgn_hdf_stage streams into HBM through two pinned buffers.
// The step kernels then read the tape in place (one cursor per env), so a
// replay env costs the same HBM reads as a generator env and the series is
// read from disk once, not per env.
#include <hdf5.h>
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/madigan_amd.h"
#include "../../include/madigan_hdf.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

struct Hid {  // scoped HDF5 identifier
  hid_t id = -1;
  herr_t (*close)(hid_t) = nullptr;
  Hid() = default;
  Hid(hid_t i, herr_t (*c)(hid_t)) : id(i), close(c) {}
  Hid(const Hid&) = delete;
  Hid& operator=(const Hid&) = delete;
  Hid& operator=(Hid&& o) noexcept {
    reset();
    id = o.id;
    close = o.close;
    o.id = -1;
    return *this;
  }
  ~Hid() { reset(); }
  void reset() {
    if (id >= 0 && close) close(id);
    id = -1;
  }
  bool ok() const { return id >= 0; }
};

void quiet() { H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr); }

std::vector<hsize_t> dims_of(hid_t dset) {
  Hid sp(H5Dget_space(dset), H5Sclose);
  const int nd = H5Sget_simple_extent_ndims(sp.id);
  std::vector<hsize_t> d(nd > 0 ? nd : 0);
  if (nd > 0) H5Sget_simple_extent_dims(sp.id, d.data(), nullptr);
  return d;
}

// rows [row0, row0+n) x all columns of a 1-D or 2-D dataset
bool read_rows(hid_t dset, hid_t memtype, uint64_t row0, uint64_t n, void* out) {
  const std::vector<hsize_t> d = dims_of(dset);
  if (d.empty() || d.size() > 2 || row0 + n > d[0]) return false;
  Hid fs(H5Dget_space(dset), H5Sclose);
  hsize_t start[2] = {row0, 0}, count[2] = {n, d.size() == 2 ? d[1] : 1};
  if (H5Sselect_hyperslab(fs.id, H5S_SELECT_SET, start, nullptr, count, nullptr) < 0) return false;
  Hid ms(H5Screate_simple((int)d.size(), count, nullptr), H5Sclose);
  return H5Dread(dset, memtype, ms.id, fs.id, H5P_DEFAULT, out) >= 0;
}

}  // namespace

struct mgn_hdf {
  Hid file, group, price, feats, ts;
  std::vector<std::string> assets;
  int64_t T = 0;
  int A = 0, F = 0, price_1d = 0;
  uint64_t first = 0, second = 0;
  uint64_t start_time = 0, end_time = 0;
};

namespace {

uint64_t ts_at(const mgn_hdf* h, uint64_t i, bool& ok) {
  uint64_t v = 0;
  ok = i < (uint64_t)h->T && read_rows(h->ts.id, H5T_NATIVE_UINT64, i, 1, &v);
  return v;
}

// binarySearchSortedHDFArray (DataSource.cpp:164-189), restated with its
// size_t arithmetic: l = 0, r = T (one past the end), at most log2(T) + 2
// probes; an exact match returns at once, otherwise the last probe is returned.
int bsearch_ts(const mgn_hdf* h, uint64_t val, uint64_t& m) {
  const uint64_t T = (uint64_t)h->T;
  int max_tries = (int)std::log2((double)T) + 2;
  uint64_t l = 0, r = T;
  m = 0;
  while (l <= r && max_tries-- > 0) {
    m = l + (r - l) / 2;
    bool ok;
    const uint64_t buf = ts_at(h, m, ok);
    if (!ok) return fail(MGN_ERR_INDEX, "timestamp search read row " + std::to_string(m) +
                                            " outside the dataset");
    if (buf == val) return MGN_OK;
    if (buf < val) l = m + 1;
    else r = m - 1;
  }
  return MGN_OK;
}

// The period of HDFSourceSingle::getData under iterCache / loadData
// (DataSource.cpp:368-408) from the state after init(): currentIdx_ = first,
// the first cache [first, first + min(cacheSize, second - first)).  Emits the
// contiguous chunks (one per cache refill) until the next refill rewinds to
// `first`.  loadData's rewind test is `currentIdx_ >= second - 1`, so a refill
// that starts at second - 1 skips that row (the period is then one row short).
void tape_chunks(const mgn_hdf* h, int64_t cache_size,
                 std::vector<std::pair<uint64_t, uint64_t>>& chunks) {
  chunks.clear();
  const uint64_t first = h->first, second = h->second;
  const uint64_t full = second - first;
  uint64_t cs = cache_size < 1 ? 1 : (uint64_t)cache_size;
  cs = std::min(cs, full);                   // loadDimsInfo, :299
  uint64_t cur = first;
  if (cur >= second - 1) cur = first;        // loadData, :369-371
  uint64_t ccs = std::min(cs, second - cur);
  chunks.emplace_back(cur, ccs);
  if (ccs >= full) return;                   // iterCache's rewind branch, :397-399
  cur += ccs;
  while (true) {
    if (cur >= second - 1) return;           // the refill rewinds: period complete
    ccs = std::min(cs, second - cur);
    chunks.emplace_back(cur, ccs);
    cur += ccs;
  }
}

}  // namespace

extern "C" {

int mgn_hdf_open(const char* path, const char* group, const char* price_key,
                 const char* feature_key, const char* timestamp_key, uint64_t start_time,
                 uint64_t end_time, mgn_hdf** out) {
  if (!out || !path || !group || !price_key || !feature_key || !timestamp_key)
    return fail(MGN_ERR_ARG, "null argument");
  *out = nullptr;
  quiet();
  auto* h = new mgn_hdf();
  auto bail = [&](int code, const std::string& m) {
    delete h;
    return fail(code, m);
  };
  h->file = Hid(H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT), H5Fclose);
  if (!h->file.ok()) return bail(MGN_ERR_CONFIG, std::string("cannot open HDF5 file ") + path);
  // checkKeys (DataSource.cpp:264-274)
  if (H5Lexists(h->file.id, group, H5P_DEFAULT) <= 0)
    return bail(MGN_ERR_CONFIG, std::string("group ") + group + " not found in hdfile: " + path);
  h->group = Hid(H5Gopen2(h->file.id, group, H5P_DEFAULT), H5Gclose);
  if (!h->group.ok()) return bail(MGN_ERR_CONFIG, std::string("cannot open group ") + group);
  if (H5Aexists(h->group.id, "assets") <= 0)
    return bail(MGN_ERR_CONFIG, std::string("key: assetsnot found in ") + group + " in hdfile: " + path);
  for (const char* k : {price_key, feature_key, timestamp_key})
    if (H5Lexists(h->group.id, k, H5P_DEFAULT) <= 0)
      return bail(MGN_ERR_CONFIG, std::string("key: ") + k + "not found in " + group +
                                      " in hdfile: " + path);
  // loadAssets (:277-285): the "assets" string attribute
  {
    Hid a(H5Aopen(h->group.id, "assets", H5P_DEFAULT), H5Aclose);
    Hid ft(H5Aget_type(a.id), H5Tclose);
    Hid sp(H5Aget_space(a.id), H5Sclose);
    const hssize_t n = H5Sget_simple_extent_npoints(sp.id);
    if (H5Tget_class(ft.id) != H5T_STRING || n < 1)
      return bail(MGN_ERR_CONFIG, "attribute assets must hold strings");
    Hid mt(H5Tcopy(H5T_C_S1), H5Tclose);
    if (H5Tis_variable_str(ft.id) > 0) {
      H5Tset_size(mt.id, H5T_VARIABLE);
      std::vector<char*> buf((size_t)n, nullptr);
      if (H5Aread(a.id, mt.id, buf.data()) < 0) return bail(MGN_ERR_CONFIG, "cannot read assets");
      for (auto* s : buf) h->assets.emplace_back(s ? s : "");
      H5Dvlen_reclaim(mt.id, sp.id, H5P_DEFAULT, buf.data());
    } else {
      const size_t w = H5Tget_size(ft.id);
      H5Tset_size(mt.id, w);
      std::vector<char> buf((size_t)n * w + 1, 0);
      if (H5Aread(a.id, mt.id, buf.data()) < 0) return bail(MGN_ERR_CONFIG, "cannot read assets");
      for (hssize_t i = 0; i < n; ++i)
        h->assets.emplace_back(std::string(buf.data() + i * w, strnlen(buf.data() + i * w, w)));
    }
  }
  h->A = (int)h->assets.size();
  if (h->A > MGN_MAX_ASSETS) return bail(MGN_ERR_LENGTH, "more than 64 assets in the file");
  h->price = Hid(H5Dopen2(h->group.id, price_key, H5P_DEFAULT), H5Dclose);
  h->feats = Hid(H5Dopen2(h->group.id, feature_key, H5P_DEFAULT), H5Dclose);
  h->ts = Hid(H5Dopen2(h->group.id, timestamp_key, H5P_DEFAULT), H5Dclose);
  if (!h->price.ok() || !h->feats.ok() || !h->ts.ok())
    return bail(MGN_ERR_CONFIG, "price/feature/timestamp keys must name datasets");
  // loadDimsInfo (:288-302): feature shape (T, F); price (T,) or (T, A)
  const auto fd = dims_of(h->feats.id), pd = dims_of(h->price.id), td = dims_of(h->ts.id);
  if (fd.empty() || fd.size() > 2 || pd.empty() || pd.size() > 2 || td.size() != 1)
    return bail(MGN_ERR_LENGTH, "datasets must be price (T,)|(T,A), features (T,F), timestamps (T,)");
  h->T = (int64_t)td[0];
  h->F = fd.size() == 2 ? (int)fd[1] : 1;
  h->price_1d = pd.size() == 1;
  if (fd[0] != td[0] || pd[0] != td[0])
    return bail(MGN_ERR_LENGTH, "price, feature and timestamp datasets differ in length");
  if ((h->price_1d && h->A != 1) || (!h->price_1d && (int)pd[1] != h->A))
    return bail(MGN_ERR_LENGTH, "price columns do not match the assets attribute");
  if (h->F < 1 || h->F > MGN_MAX_ASSETS) return bail(MGN_ERR_LENGTH, "n_feats must be in [1, 64]");
  if (h->T < 1) return bail(MGN_ERR_LENGTH, "empty timestamp dataset");
  // getTimeBounds (:305-322) with getBounds (:145-160)
  bool ok0, ok1;
  const uint64_t b0 = ts_at(h, 0, ok0), b1 = ts_at(h, (uint64_t)h->T - 1, ok1);
  if (!ok0 || !ok1) return bail(MGN_ERR_CONFIG, "cannot read timestamps");
  if (start_time == 0 && end_time == 0) {
    start_time = b0;
    end_time = b1;
  } else if (!(start_time >= b0 && end_time <= b1)) {
    return bail(MGN_ERR_INDEX, "Given start and endTimes not within bounds found in timestamp data");
  }
  h->start_time = start_time;
  h->end_time = end_time;
  // findBounds (:324-366)
  uint64_t si, ei;
  int rc = bsearch_ts(h, start_time, si);
  if (rc == MGN_OK) rc = bsearch_ts(h, end_time, ei);
  if (rc != MGN_OK) {
    const std::string m = g_err;
    return bail(rc, m);
  }
  if (ei - si < 2)
    return bail(MGN_ERR_LENGTH, "dset size only " + std::to_string(ei - si) + " !");
  bool ok;
  uint64_t buf = ts_at(h, si, ok);
  if (!ok) return bail(MGN_ERR_INDEX, "start index outside the dataset");
  if (buf == start_time || si == 0) h->first = si;
  else h->first = (buf < start_time) ? si + 1 : si;
  buf = ts_at(h, ei, ok);
  if (!ok) return bail(MGN_ERR_INDEX, "end index outside the dataset");
  if (buf == end_time || ei == (uint64_t)h->T - 1) h->second = ei;
  else h->second = (buf > end_time) ? ei - 1 : ei;  // end not included
  // an empty or inverted bounded range makes the reference read an empty cache
  // (undefined behaviour); here it is a length error
  if (h->second <= h->first || h->second > (uint64_t)h->T)
    return bail(MGN_ERR_LENGTH, "no rows between the time bounds");
  *out = h;
  return MGN_OK;
}

int mgn_hdf_close(mgn_hdf* h) {
  delete h;
  return MGN_OK;
}

int mgn_hdf_get_info(const mgn_hdf* h, mgn_hdf_info* info) {
  if (!h || !info) return fail(MGN_ERR_ARG, "null handle/info");
  info->n_rows = h->T;
  info->n_assets = h->A;
  info->n_feats = h->F;
  info->first = (int64_t)h->first;
  info->second = (int64_t)h->second;
  info->start_time = h->start_time;
  info->end_time = h->end_time;
  info->price_1d = h->price_1d;
  info->pad_ = 0;
  return MGN_OK;
}

int mgn_hdf_asset(const mgn_hdf* h, int32_t i, char* buf, size_t len) {
  if (!h || !buf || len == 0) return fail(MGN_ERR_ARG, "null handle/buffer");
  if (i < 0 || i >= h->A) return fail(MGN_ERR_INDEX, "asset index out of range");
  const std::string& s = h->assets[(size_t)i];
  const size_t n = std::min(len - 1, s.size());
  memcpy(buf, s.data(), n);
  buf[n] = 0;
  return MGN_OK;
}

int mgn_hdf_read(const mgn_hdf* h, int64_t row0, int64_t n, double* price, double* feats,
                 uint64_t* ts) {
  if (!h) return fail(MGN_ERR_ARG, "null handle");
  if (row0 < 0 || n < 0 || row0 + n > h->T) return fail(MGN_ERR_INDEX, "rows outside the dataset");
  if (n == 0) return MGN_OK;
  if (price && !read_rows(h->price.id, H5T_NATIVE_DOUBLE, (uint64_t)row0, (uint64_t)n, price))
    return fail(MGN_ERR_CONFIG, "cannot read price rows");
  if (feats && !read_rows(h->feats.id, H5T_NATIVE_DOUBLE, (uint64_t)row0, (uint64_t)n, feats))
    return fail(MGN_ERR_CONFIG, "cannot read feature rows");
  if (ts && !read_rows(h->ts.id, H5T_NATIVE_UINT64, (uint64_t)row0, (uint64_t)n, ts))
    return fail(MGN_ERR_CONFIG, "cannot read timestamp rows");
  return MGN_OK;
}

int64_t mgn_hdf_tape_rows(const mgn_hdf* h, int64_t cache_size) {
  if (!h) return -1;
  std::vector<std::pair<uint64_t, uint64_t>> ch;
  tape_chunks(h, cache_size, ch);
  int64_t n = 0;
  for (auto& c : ch) n += (int64_t)c.second;
  return n;
}

int mgn_hdf_tape_index(const mgn_hdf* h, int64_t cache_size, int64_t* rows) {
  if (!h || !rows) return fail(MGN_ERR_ARG, "null handle/rows");
  std::vector<std::pair<uint64_t, uint64_t>> ch;
  tape_chunks(h, cache_size, ch);
  int64_t j = 0;
  for (auto& c : ch)
    for (uint64_t r = 0; r < c.second; ++r) rows[j++] = (int64_t)(c.first + r);
  return MGN_OK;
}

int mgn_hdf_stage(const mgn_hdf* h, int64_t cache_size, double* price_dev, double* feats_dev,
                  uint64_t* ts_dev, uint8_t* data_end_dev, void* stream_) {
  if (!h || !price_dev || !feats_dev || !ts_dev || !data_end_dev)
    return fail(MGN_ERR_ARG, "null handle/device pointer");
  hipStream_t stream = (hipStream_t)stream_;
  std::vector<std::pair<uint64_t, uint64_t>> ch;
  tape_chunks(h, cache_size, ch);
  // staging pieces: the refill chunks, split to at most 256 Ki rows
  constexpr uint64_t MAXR = 1u << 18;
  std::vector<std::pair<uint64_t, uint64_t>> pieces;
  for (auto& c : ch)
    for (uint64_t o = 0; o < c.second; o += MAXR)
      pieces.emplace_back(c.first + o, std::min(MAXR, c.second - o));
  uint64_t maxr = 0;
  for (auto& p : pieces) maxr = std::max(maxr, p.second);
  const size_t A = (size_t)h->A, F = (size_t)h->F;
  const size_t slot = maxr * (8 * (A + F) + 8 + 1);
  void* pin[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  int rc = MGN_OK;
  for (int b = 0; b < 2 && rc == MGN_OK; ++b) {
    if (hipHostMalloc(&pin[b], slot, hipHostMallocDefault) != hipSuccess)
      rc = fail(MGN_ERR_DEVICE, "hipHostMalloc of the staging buffers failed");
    else if (hipEventCreateWithFlags(&ev[b], hipEventDisableTiming) != hipSuccess)
      rc = fail(MGN_ERR_DEVICE, "hipEventCreate failed");
  }
  uint64_t off = 0;
  for (size_t i = 0; i < pieces.size() && rc == MGN_OK; ++i) {
    const int b = (int)(i & 1);
    // the copy that last used this buffer must have drained before it is refilled;
    // meanwhile the other buffer's copy is in flight
    if (i >= 2 && hipEventSynchronize(ev[b]) != hipSuccess) {
      rc = fail(MGN_ERR_DEVICE, "hipEventSynchronize failed");
      break;
    }
    const uint64_t r0 = pieces[i].first, n = pieces[i].second;
    char* base = (char*)pin[b];
    double* pp = (double*)base;
    double* pf = pp + n * A;
    uint64_t* pt = (uint64_t*)(pf + n * F);
    uint8_t* pe = (uint8_t*)(pt + n);
    rc = mgn_hdf_read(h, (int64_t)r0, (int64_t)n, pp, pf, pt);
    if (rc != MGN_OK) break;
    for (uint64_t r = 0; r < n; ++r) pe[r] = (r0 + r + 1 == h->second) ? 1 : 0;  // dataEnd()
    hipError_t e = hipMemcpyAsync(price_dev + off * A, pp, n * A * 8, hipMemcpyHostToDevice, stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(feats_dev + off * F, pf, n * F * 8, hipMemcpyHostToDevice, stream);
    if (e == hipSuccess) e = hipMemcpyAsync(ts_dev + off, pt, n * 8, hipMemcpyHostToDevice, stream);
    if (e == hipSuccess) e = hipMemcpyAsync(data_end_dev + off, pe, n, hipMemcpyHostToDevice, stream);
    if (e == hipSuccess) e = hipEventRecord(ev[b], stream);
    if (e != hipSuccess) rc = fail(MGN_ERR_DEVICE, std::string("H2D staging: ") + hipGetErrorString(e));
    off += n;
  }
  if (hipStreamSynchronize(stream) != hipSuccess && rc == MGN_OK)
    rc = fail(MGN_ERR_DEVICE, "hipStreamSynchronize failed");
  for (int b = 0; b < 2; ++b) {
    if (ev[b]) (void)hipEventDestroy(ev[b]);
    if (pin[b]) (void)hipHostFree(pin[b]);
  }
  return rc;
}

int mgn_hdf_write(const char* path, const char* group, const char* price_key,
                  const char* feature_key, const char* timestamp_key, const char* const* assets,
                  int32_t n_assets, int64_t n_rows, int32_t n_feats, const double* price,
                  const double* feats, const uint64_t* ts, int32_t price_1d) {
  if (!path || !group || !price_key || !feature_key || !timestamp_key || !assets || !price ||
      !feats || !ts)
    return fail(MGN_ERR_ARG, "null argument");
  if (n_assets < 1 || n_rows < 1 || n_feats < 1 || (price_1d && n_assets != 1))
    return fail(MGN_ERR_LENGTH, "bad dimensions");
  quiet();
  Hid f(H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT), H5Fclose);
  if (!f.ok()) return fail(MGN_ERR_CONFIG, std::string("cannot create ") + path);
  Hid lcpl(H5Pcreate(H5P_LINK_CREATE), H5Pclose);
  H5Pset_create_intermediate_group(lcpl.id, 1);  // "group/dataset" -> nested groups
  Hid g(H5Gcreate2(f.id, group, lcpl.id, H5P_DEFAULT, H5P_DEFAULT), H5Gclose);
  if (!g.ok()) return fail(MGN_ERR_CONFIG, std::string("cannot create group ") + group);
  {
    hsize_t n = (hsize_t)n_assets;
    Hid sp(H5Screate_simple(1, &n, nullptr), H5Sclose);
    Hid st(H5Tcopy(H5T_C_S1), H5Tclose);
    H5Tset_size(st.id, H5T_VARIABLE);
    Hid a(H5Acreate2(g.id, "assets", st.id, sp.id, H5P_DEFAULT, H5P_DEFAULT), H5Aclose);
    if (!a.ok() || H5Awrite(a.id, st.id, assets) < 0)
      return fail(MGN_ERR_CONFIG, "cannot write the assets attribute");
  }
  auto put = [&](const char* key, hid_t type, int nd, hsize_t d0, hsize_t d1, const void* data) {
    hsize_t d[2] = {d0, d1};
    Hid sp(H5Screate_simple(nd, d, nullptr), H5Sclose);
    Hid ds(H5Dcreate2(g.id, key, type, sp.id, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT), H5Dclose);
    return ds.ok() && H5Dwrite(ds.id, type, H5S_ALL, H5S_ALL, H5P_DEFAULT, data) >= 0;
  };
  const hsize_t T = (hsize_t)n_rows;
  if (!put(price_key, H5T_NATIVE_DOUBLE, price_1d ? 1 : 2, T, (hsize_t)n_assets, price) ||
      !put(feature_key, H5T_NATIVE_DOUBLE, 2, T, (hsize_t)n_feats, feats) ||
      !put(timestamp_key, H5T_NATIVE_UINT64, 1, T, 0, ts))
    return fail(MGN_ERR_CONFIG, "cannot write datasets");
  return MGN_OK;
}

const char* mgn_hdf_last_error(void) { return g_err.c_str(); }

}  // extern "C"
