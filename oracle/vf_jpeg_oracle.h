/* vf_jpeg_oracle.h — CPU ORACLE, TEST INFRASTRUCTURE ONLY (see vf_jpeg_oracle.c). */
#ifndef VF_JPEG_ORACLE_H
#define VF_JPEG_ORACLE_H

#include <stddef.h>
#include <stdint.h>

/* TurboJPEG constants (turbojpeg.h), as PyTurboJPEG exposes them */
#define VFO_SAMP_444 0
#define VFO_SAMP_422 1
#define VFO_SAMP_420 2
#define VFO_SAMP_GRAY 3
#define VFO_SAMP_440 4
#define VFO_PF_RGB 0
#define VFO_PF_BGR 1

#define VFO_JE_OK 0
#define VFO_JE_NOT_JPEG -1
#define VFO_JE_TRUNCATED -2
#define VFO_JE_BAD -3
#define VFO_JE_UNSUPPORTED -4
#define VFO_JE_NOMEM -5
#define VFO_JE_ARG -6

typedef struct {
  int width, height, ncomp;
  int comp_id[3], h[3], v[3], tq[3], td[3], ta[3];
  int max_h, max_v;
  int restart_interval;
  uint16_t qt[4][64]; /* natural order */
  int qt_defined, dc_defined, ac_defined;
  uint8_t dc_bits[4][17], ac_bits[4][17];
  uint8_t dc_vals[4][256], ac_vals[4][256];
  size_t scan_offset, scan_end; /* entropy-coded segment [scan_offset, scan_end) */
} vfo_jpeg_info;

int vfo_jpeg_quality_table(int quality, int chroma, uint16_t out[64]);
void vfo_jpeg_divisors(const uint16_t q[64], int fastdct, uint16_t recip[64], uint16_t corr[64],
                       int16_t shift[64]);
void vfo_fdct_islow(int32_t d[64]);
void vfo_fdct_ifast(int32_t d[64]);
void vfo_idct_islow(const int16_t coef[64], const uint16_t q[64], uint8_t *out, int stride);
void vfo_huff_encode_table(const uint8_t bits[17], const uint8_t *vals, uint16_t code[256],
                           uint8_t size[256]);
size_t vfo_jpeg_write_headers(int w, int h, int quality, int subsamp, uint8_t *out, size_t cap);
size_t vfo_jpeg_encode(const uint8_t *img, int w, int h, int pixel_format, int quality,
                       int subsamp, int fastdct, uint8_t *out, size_t cap);
size_t vfo_jpeg_encode_bound(int w, int h, int subsamp);
int vfo_jpeg_parse(const uint8_t *jpg, size_t n, vfo_jpeg_info *info);
int vfo_jpeg_decode(const uint8_t *jpg, size_t n, int pixel_format, int fast_upsample, uint8_t *out,
                    size_t cap);

#endif
