/* liteasr_io.h -- native Kaldi feature reader of the MI355X LiteASR training path.
 *
 * Host-side C ABI (libliteasr_io.so, plain C++17, no device code): decodes the Kaldi binary
 * matrices that feats.scp entries point at ("<ark>:<byte offset>") straight into caller-owned
 * (typically pinned) buffers, so the collated batch can be copied to HBM with one DMA.
 *
 * Replaces (reference, Python):
 *   liteasr/utils/kaldiio/matio.py:225-241   load_mat(ark_name)          -> lasr_ark_probe + lasr_ark_read
 *   liteasr/utils/kaldiio/matio.py:371-443   read_kaldi (binary "\0B")   -> same
 *   liteasr/utils/kaldiio/matio.py:460-554   read_matrix_or_vector       -> FM/FV/DM/DV/CM/CM2/CM3 decode
 *   liteasr/utils/kaldiio/compression_header.py:17-251 (GlobalHeader / PerColHeader decode)
 *   liteasr/dataset/asr_dataset.py:115-126   collator: pad_sequence(xs, batch_first, 0)
 *                                            -> lasr_ark_read_padded
 *
 * Conventions: 0 = success, negative = error (message in lasr_io_last_error(), thread-local).
 * Decoded values are bit-identical to the reference's numpy float32 arithmetic.
 */
#ifndef LITEASR_IO_H
#define LITEASR_IO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* storage kinds of a Kaldi binary object */
enum {
  LASR_ARK_FM = 1,  /* float matrix            */
  LASR_ARK_FV = 2,  /* float vector            */
  LASR_ARK_DM = 3,  /* double matrix           */
  LASR_ARK_DV = 4,  /* double vector           */
  LASR_ARK_CM = 5,  /* compressed, per-column 8-bit (kSpeechFeature) */
  LASR_ARK_CM2 = 6, /* compressed, global 16-bit */
  LASR_ARK_CM3 = 7  /* compressed, global 8-bit  */
};

/* output element types for lasr_ark_read */
enum { LASR_IO_F32 = 0, LASR_IO_F64 = 1 };

int lasr_io_version(void);
const char* lasr_io_last_error(void);

/* Header of the object at (path, offset): rows, cols (vectors: rows = length, cols = 0),
 * kind.  big_endian != 0 reads a '>' ark.  offset < 0 reads from the start of the file. */
int lasr_ark_probe(const char* path, int64_t offset, int big_endian, int64_t* rows,
                   int64_t* cols, int* kind);

/* Decode the object into out (row-major, row stride ld elements, at most max_rows rows are
 * written; vectors are one row).  out_dtype LASR_IO_F32 or LASR_IO_F64. */
int lasr_ark_read(const char* path, int64_t offset, int big_endian, void* out, int out_dtype,
                  int64_t max_rows, int64_t ld, int64_t* rows, int64_t* cols);

/* Collate n feature matrices into out[n][tmax][feat_dim] float32 (zero padded, the
 * reference collator's pad_sequence(batch_first=True, padding_value=0)); lens[i] receives
 * the frame count of matrix i.  Every matrix must have feat_dim columns and at most tmax
 * rows.  Decoding runs on nthreads host threads (<= 0: one per hardware thread, max 16). */
int lasr_ark_read_padded(int n, const char* const* paths, const int64_t* offsets, int big_endian,
                         float* out, int64_t tmax, int64_t feat_dim, int64_t* lens, int nthreads);

#ifdef __cplusplus
}
#endif

#endif /* LITEASR_IO_H */
