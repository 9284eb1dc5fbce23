/*
 * madigan_hdf.h -- HDF replay DataSource: reader, fixture writer and the
 * host-pinned, double-buffered H2D staging of the replay tape
 * (libmadigan_hdf.so; host code over libhdf5 and the HIP runtime).
 *
 * Replaces the reference's HDFSourceSingle (madigan/environments/cpp/
 * DataSource.h:89-149, DataSource.cpp:194-408) on the MI355X path:
 *   mgn_hdf_open     HDFSourceSingle(filepath, groupKey, priceKey, featureKey,
 *                    timestampKey, cacheSize[, startTime, endTime]) -- the
 *                    init() chain checkKeys / loadAssets / loadDimsInfo /
 *                    getTimeBounds / findBounds (DataSource.cpp:194-366)
 *   mgn_hdf_read     loadVectorFromHDF / loadMatrixFromHDF (DataSource.cpp:127-162)
 *   mgn_hdf_tape_*   the row sequence HDFSourceSingle::getData visits under
 *                    iterCache / loadData (DataSource.cpp:368-408), one period
 *   mgn_hdf_stage    that period streamed into device memory chunk by chunk
 *                    (the reference's cache refills) through two pinned host
 *                    buffers: the HDF read of chunk i+1 overlaps the H2D copy
 *                    of chunk i
 *   mgn_hdf_write    the fixture writer of envTest.cpp:322-368 (layout: group
 *                    attribute "assets" (strings), datasets price (T,) or (T,A),
 *                    features (T,F), timestamps uint64 (T,))
 *
 * Layout generalisation: price may be (T, A) with A = number
 * of asset codes in the "assets" attribute (HDFSourceMulti is declared but not
 * defined in the reference, DataSource.h:154-185); (T,) is the A = 1 case.
 *
 * Errors: MGN_ERR_CONFIG = ConfigError (missing key / attribute), MGN_ERR_INDEX
 * = std::out_of_range (time bounds outside the data), MGN_ERR_LENGTH =
 * std::length_error (fewer than 2 rows in bounds, shape mismatch); the text is
 * in mgn_hdf_last_error().
 */
#ifndef MADIGAN_HDF_H_
#define MADIGAN_HDF_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mgn_hdf mgn_hdf;

typedef struct {
  int64_t n_rows;        /* T: rows in the file */
  int32_t n_assets;      /* entries of the "assets" attribute */
  int32_t n_feats;       /* F: columns of the feature dataset */
  int64_t first, second; /* boundsIdx_ (DataSource.cpp:338-366); rows [first, second) */
  uint64_t start_time, end_time; /* startTime / endTime after getTimeBounds */
  int32_t price_1d;      /* price dataset is (T,) */
  int32_t pad_;
} mgn_hdf_info;

/* start_time == end_time == 0: bounds from the data (DataSource.cpp:307-322) */
int mgn_hdf_open(const char *path, const char *group, const char *price_key,
                 const char *feature_key, const char *timestamp_key, uint64_t start_time,
                 uint64_t end_time, mgn_hdf **out);
int mgn_hdf_close(mgn_hdf *h);
int mgn_hdf_get_info(const mgn_hdf *h, mgn_hdf_info *info);
/* asset code i into buf (NUL-terminated, truncated to len) */
int mgn_hdf_asset(const mgn_hdf *h, int32_t i, char *buf, size_t len);
/* rows [row0, row0+n) into host arrays price (n,A), feats (n,F), ts (n); any may be NULL */
int mgn_hdf_read(const mgn_hdf *h, int64_t row0, int64_t n, double *price, double *feats,
                 uint64_t *ts);
/* rows of one period of getData's visiting order for cache_size (cacheSize,
 * DataSource.cpp:235, clamped to the bounded length as :299) */
int64_t mgn_hdf_tape_rows(const mgn_hdf *h, int64_t cache_size);
/* that period's file row indices (host, n = mgn_hdf_tape_rows) */
int mgn_hdf_tape_index(const mgn_hdf *h, int64_t cache_size, int64_t *rows);
/* stream the period into device arrays: price (P,A), feats (P,F), ts (P),
 * data_end (P) (= HDFSourceSingle::dataEnd() after that getData, DataSource.h:126),
 * on `stream` (hipStream_t, NULL = null stream); returns after the last copy */
int mgn_hdf_stage(const mgn_hdf *h, int64_t cache_size, double *price_dev, double *feats_dev,
                  uint64_t *ts_dev, uint8_t *data_end_dev, void *stream);
/* fixture writer; price is (T,) when price_1d (requires n_assets == 1), else (T, n_assets) */
int mgn_hdf_write(const char *path, const char *group, const char *price_key,
                  const char *feature_key, const char *timestamp_key, const char *const *assets,
                  int32_t n_assets, int64_t n_rows, int32_t n_feats, const double *price,
                  const double *feats, const uint64_t *ts, int32_t price_1d);
const char *mgn_hdf_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
