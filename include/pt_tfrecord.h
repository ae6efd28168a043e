/*
 * pt_tfrecord.h — C ABI of the native PathTracker clip reader / writer
 * (libpttfr.so, host C++, zlib).
 *
 * Replaces the reference's TensorFlow input pipeline (utils/TFRDataset.py):
 *   read_tfrecord      :6-28   parse one tf.train.Example: 'image' bytes
 *                              (T x 32 x 32 x 3 uint8, decode_raw + reshape),
 *                              'label' bytes; 'height' / 'width' int64 unused
 *   tfr_data_loader    :31-53  glob -> TFRecordDataset(GZIP) -> map(parse) ->
 *                              shuffle(buffer) -> batch(B, drop_remainder)
 * with per-rank file sharding for one-process-per-GPU training (file i goes
 * to rank i % world: each rank reads disjoint shards, no scatter).
 *
 * Record framing (TFRecord): u64 length (LE), u32 masked crc32c(length),
 * length bytes of data, u32 masked crc32c(data); masked(c) =
 * ((c >> 15) | (c << 17)) + 0xa282ead8.  Files are gzip streams (TF's
 * compression_type='GZIP').
 *
 * Conventions: plain C types; the caller owns every output buffer; int / int64
 * status (< 0 = error) with a thread-local message from pt_tfr_last_error().
 * A reader handle is used from one host thread at a time; it runs its own
 * decoder threads internally.
 */
#ifndef PT_TFRECORD_H
#define PT_TFRECORD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { PT_TFR_OK = 0, PT_TFR_ERR_ARG = -1, PT_TFR_ERR_IO = -2, PT_TFR_ERR_FORMAT = -3 };

typedef struct pt_tfr_options {
    int32_t timesteps;       /* T (reshape [T, H, W, C], TFRDataset.py:20)          */
    int32_t height;          /* H (32)                                               */
    int32_t width;           /* W (32)                                               */
    int32_t channels;        /* C (3)                                                */
    int32_t rank;            /* this process's rank                                  */
    int32_t world;           /* number of ranks; file i is read by rank i % world   */
    int32_t shuffle_buffer;  /* 0: file order; else tf.data shuffle(buffer) sampling */
    int32_t threads;         /* decoder threads (>= 1)                               */
    int32_t verify_crc;      /* check both masked CRCs of every record               */
    int32_t drop_remainder;  /* batch(B, drop_remainder), TFRDataset.py:52           */
    uint64_t seed;           /* shuffle seed                                         */
} pt_tfr_options;

typedef struct pt_tfr_reader pt_tfr_reader;

/* Open a reader over `npaths` files (the caller's glob, in the order given).
 * Returns NULL on error. */
pt_tfr_reader* pt_tfr_open(const char* const* paths, int32_t npaths, const pt_tfr_options* o);

/* Next batch: fills clips [batch][T][H][W][C] uint8 and labels [batch] (the
 * single byte of each 'label' string, what engine.prepare_data ord()s).
 * Returns the number of clips written: `batch`, a short final batch (only
 * without drop_remainder), 0 at the end of the data, or < 0 on error. */
int64_t pt_tfr_next(pt_tfr_reader* r, int32_t batch, uint8_t* clips, uint8_t* labels);

/* Records this reader has produced so far, and closing. */
int64_t pt_tfr_count(const pt_tfr_reader* r);
int pt_tfr_close(pt_tfr_reader* r);

/* Write n clips [n][T][H][W][C] with their label bytes as one TFRecord file of
 * tf.train.Example records {'height', 'image', 'label', 'width'} (gzip when
 * `gzip` != 0).  The synthetic-data generator and the tests use this. */
int pt_tfr_write(const char* path, const uint8_t* clips, const uint8_t* labels, int64_t n,
                 int32_t t, int32_t h, int32_t w, int32_t c, int32_t gzip);

/* One serialized tf.train.Example -> its 'image' bytes (copied into `image`,
 * capacity image_cap) and the single 'label' byte (read_tfrecord,
 * TFRDataset.py:6-28).  Returns the image byte count or < 0. */
int64_t pt_tfr_parse_example(const uint8_t* data, size_t n, uint8_t* image, size_t image_cap,
                             uint8_t* label);

/* CRC32C (Castagnoli) and TFRecord's masked form. */
uint32_t pt_tfr_crc32c(const uint8_t* data, size_t n);
uint32_t pt_tfr_masked_crc32c(const uint8_t* data, size_t n);

const char* pt_tfr_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PT_TFRECORD_H */
