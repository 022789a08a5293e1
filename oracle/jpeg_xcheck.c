/*
 * jpeg_xcheck.c — TEST INFRASTRUCTURE ONLY.
 *
 * Runs the image's libjpeg-turbo (libjpeg.so.8 = libjpeg-turbo 2.1.2, the codec that
 * libturbojpeg wraps under PyTurboJPEG, inverter.py:13,32,44) the way TurboJPEG drives it,
 * so tests can cross-check the restatement in vf_jpeg_oracle.c and generate golden vectors.
 * It is a checker: nothing in the product links or loads it.
 *
 * The image ships the library but not its headers, so the libjpeg v8 API subset used here
 * is declared below from the public jpeglib.h interface.  Every struct offset this file
 * touches is verified at run time against values libjpeg itself writes:
 * jpeg_CreateCompress / jpeg_CreateDecompress reject a wrong struct size (the decompress
 * size is probed that way), jpeg_set_defaults and jpeg_read_header fill known fields, and
 * xc_encode / xc_decode refuse to run if any check fails.
 *
 * Mirrors turbojpeg.c (2.1.x): tjCompress2 -> setCompDefaults (jpeg_set_defaults,
 * jpeg_set_quality(q, TRUE), dct_method, jpeg_set_colorspace, per-TJSAMP sampling) and
 * tjDecompress2 -> setDecompDefaults (out_color_space, fancy upsampling, dct_method).
 */
#include <dlfcn.h>
#include <setjmp.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define JPEG_LIB_VERSION 80
#define JCS_GRAYSCALE 1
#define JCS_RGB 2
#define JCS_YCbCr 3
#define JCS_EXT_BGR 8
#define JDCT_ISLOW 0
#define JDCT_IFAST 1

/* struct jpeg_compress_struct (jpeglib.h, JPEG_LIB_VERSION 80, boolean = int) */
typedef struct {
  void *err, *mem, *progress, *client_data;
  int is_decompressor, global_state;
  void *dest;
  unsigned image_width, image_height;
  int input_components, in_color_space;
  double input_gamma;
  unsigned scale_num, scale_denom, jpeg_width, jpeg_height;
  int data_precision, num_components, jpeg_color_space;
  char *comp_info;
  void *quant_tbl_ptrs[4];
  int q_scale_factor[4];
  void *dc_huff_tbl_ptrs[4], *ac_huff_tbl_ptrs[4];
  unsigned char arith_dc_L[16], arith_dc_U[16], arith_ac_K[16];
  int num_scans;
  const void *scan_info;
  int raw_data_in, arith_code, optimize_coding, CCIR601_sampling, do_fancy_downsampling;
  int smoothing_factor, dct_method;
  unsigned restart_interval;
  int restart_in_rows, write_JFIF_header;
  unsigned char JFIF_major_version, JFIF_minor_version, density_unit;
  unsigned short X_density, Y_density;
  int write_Adobe_marker;
  unsigned next_scanline;
  int progressive_mode, max_h_samp_factor, max_v_samp_factor;
  int min_DCT_h_scaled_size, min_DCT_v_scaled_size;
  unsigned total_iMCU_rows;
  int comps_in_scan;
  void *cur_comp_info[4];
  unsigned MCUs_per_row, MCU_rows_in_scan;
  int blocks_in_MCU, MCU_membership[10], Ss, Se, Ah, Al, block_size;
  const int *natural_order;
  int lim_Se;
  void *master, *main, *prep, *coef, *marker, *cconvert, *downsample, *fdct, *entropy;
  void *script_space;
  int script_space_size;
} cinfo_t;

#define COMP_INFO_SIZE 96 /* sizeof(jpeg_component_info): 21 ints/unsigned + 2 pointers */
/* struct jpeg_decompress_struct offsets used (checked after jpeg_read_header) */
#define D_IMAGE_WIDTH 48
#define D_IMAGE_HEIGHT 52
#define D_NUM_COMPONENTS 56
#define D_JPEG_COLOR_SPACE 60
#define D_OUT_COLOR_SPACE 64
#define D_SCALE_NUM 68
#define D_SCALE_DENOM 72
#define D_DCT_METHOD 96
#define D_DO_FANCY_UPSAMPLING 100

static void *(*p_std_error)(void *);
static void (*p_CreateCompress)(void *, int, size_t);
static void (*p_CreateDecompress)(void *, int, size_t);
static void (*p_mem_dest)(void *, unsigned char **, unsigned long *);
static void (*p_mem_src)(void *, const unsigned char *, unsigned long);
static void (*p_set_defaults)(void *);
static void (*p_set_quality)(void *, int, int);
static void (*p_set_colorspace)(void *, int);
static void (*p_start_compress)(void *, int);
static unsigned (*p_write_scanlines)(void *, unsigned char **, unsigned);
static void (*p_finish_compress)(void *);
static void (*p_destroy)(void *);
static int (*p_read_header)(void *, int);
static int (*p_start_decompress)(void *);
static unsigned (*p_read_scanlines)(void *, unsigned char **, unsigned);
static int (*p_finish_decompress)(void *);

static int g_state = 0; /* 0 = not loaded, 1 = ready, -1 = unavailable */
static char g_why[256] = "not loaded";
static size_t g_dsize = 0;
static jmp_buf g_jmp;
static char g_errmgr[1024] __attribute__((aligned(16))); /* struct jpeg_error_mgr storage */
static char g_msg[128];

static void on_error_exit(void *cinfo) {
  (void)cinfo;
  /* jpeg_error_mgr: error_exit, emit_message, output_message, format_message,
   * reset_error_mgr (5 pointers), then int msg_code */
  snprintf(g_msg, sizeof g_msg, "libjpeg error code %d", *(int *)(g_errmgr + 40));
  longjmp(g_jmp, 1);
}

static void on_emit_message(void *cinfo, int level) { (void)cinfo; (void)level; }

static void *new_err(void) {
  memset(g_errmgr, 0, sizeof g_errmgr);
  void *e = p_std_error(g_errmgr);
  ((void (**)(void *))g_errmgr)[0] = on_error_exit;
  ((void (**)(void *, int))g_errmgr)[1] = on_emit_message; /* silence warnings */
  return e;
}

#define SYM(v, name)                                   \
  do {                                                 \
    *(void **)&(v) = dlsym(h, name);                   \
    if (!(v)) {                                        \
      snprintf(g_why, sizeof g_why, "missing %s", name); \
      return -1;                                       \
    }                                                  \
  } while (0)

static int load(void) {
  void *h = dlopen("libjpeg.so.8", RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    snprintf(g_why, sizeof g_why, "dlopen libjpeg.so.8: %s", dlerror());
    return -1;
  }
  SYM(p_std_error, "jpeg_std_error");
  SYM(p_CreateCompress, "jpeg_CreateCompress");
  SYM(p_CreateDecompress, "jpeg_CreateDecompress");
  SYM(p_mem_dest, "jpeg_mem_dest");
  SYM(p_mem_src, "jpeg_mem_src");
  SYM(p_set_defaults, "jpeg_set_defaults");
  SYM(p_set_quality, "jpeg_set_quality");
  SYM(p_set_colorspace, "jpeg_set_colorspace");
  SYM(p_start_compress, "jpeg_start_compress");
  SYM(p_write_scanlines, "jpeg_write_scanlines");
  SYM(p_finish_compress, "jpeg_finish_compress");
  SYM(p_destroy, "jpeg_destroy");
  SYM(p_read_header, "jpeg_read_header");
  SYM(p_start_decompress, "jpeg_start_decompress");
  SYM(p_read_scanlines, "jpeg_read_scanlines");
  SYM(p_finish_decompress, "jpeg_finish_decompress");
  /* the compress struct mirror must have the library's size */
  {
    cinfo_t c;
    memset(&c, 0, sizeof c);
    c.err = new_err();
    if (setjmp(g_jmp)) {
      snprintf(g_why, sizeof g_why, "jpeg_CreateCompress rejected the struct mirror (%zu B): %s",
               sizeof c, g_msg);
      return -1;
    }
    p_CreateCompress(&c, JPEG_LIB_VERSION, sizeof c);
    p_destroy(&c);
  }
  /* probe sizeof(struct jpeg_decompress_struct) */
  static char dbuf[4096] __attribute__((aligned(16)));
  for (volatile size_t s = 400; s <= 2048 && !g_dsize; s += 8) {
    memset(dbuf, 0, sizeof dbuf);
    *(void **)dbuf = new_err();
    if (setjmp(g_jmp) == 0) {
      p_CreateDecompress(dbuf, JPEG_LIB_VERSION, s);
      g_dsize = s;
      p_destroy(dbuf);
    }
  }
  if (!g_dsize) {
    snprintf(g_why, sizeof g_why, "could not determine sizeof(jpeg_decompress_struct)");
    return -1;
  }
  snprintf(g_why, sizeof g_why, "ok (compress %zu B, decompress %zu B)", sizeof(cinfo_t), g_dsize);
  return 1;
}

/* 1 if libjpeg.so.8 is usable, else 0; `why` (may be NULL) explains. */
int xc_available(char *why, size_t why_len) {
  if (g_state == 0) g_state = load();
  if (why && why_len) snprintf(why, why_len, "%s", g_why);
  return g_state == 1;
}

/* tjCompress2(pixel_format, subsamp TJSAMP_*, quality, flags -> dct) through libjpeg.
 * Returns the JPEG size (0 on failure or if it does not fit `cap`). */
size_t xc_encode_ex(const uint8_t *img, int w, int h, int bgr, int quality, int subsamp, int fastdct,
                    int restart_interval, int restart_in_rows, int optimize, uint8_t *out, size_t cap);

size_t xc_encode(const uint8_t *img, int w, int h, int bgr, int quality, int subsamp, int fastdct,
                 uint8_t *out, size_t cap) {
  return xc_encode_ex(img, w, h, bgr, quality, subsamp, fastdct, 0, 0, 0, out, cap);
}

/* xc_encode plus libjpeg options TurboJPEG does not set: restart_interval (MCUs) or
 * restart_in_rows (MCU rows) -> DRI + RSTn markers (jcmarker.c / jchuff.c emit_restart), and
 * optimize_coding -> per-image Huffman tables (jchuff.c jpeg_gen_optimal_table). */
size_t xc_encode_ex(const uint8_t *img, int w, int h, int bgr, int quality, int subsamp, int fastdct,
                    int restart_interval, int restart_in_rows, int optimize, uint8_t *out, size_t cap) {
  static const int samp_h[5] = {1, 2, 2, 1, 1}, samp_v[5] = {1, 1, 2, 1, 2};
  if (!xc_available(NULL, 0) || subsamp < 0 || subsamp > 4) return 0;
  cinfo_t c;
  memset(&c, 0, sizeof c);
  c.err = new_err();
  unsigned char *buf = NULL;
  unsigned long size = 0;
  size_t result = 0;
  if (setjmp(g_jmp)) {
    p_destroy(&c);
    free(buf);
    return 0;
  }
  p_CreateCompress(&c, JPEG_LIB_VERSION, sizeof c);
  p_mem_dest(&c, &buf, &size);
  c.image_width = (unsigned)w;
  c.image_height = (unsigned)h;
  c.input_components = 3;
  c.in_color_space = bgr ? JCS_EXT_BGR : JCS_RGB;
  p_set_defaults(&c);
  /* verify the mirror against what jpeg_set_defaults wrote */
  if (c.data_precision != 8 || c.num_components != 3 || c.jpeg_color_space != JCS_YCbCr ||
      c.write_JFIF_header != 1 || c.JFIF_major_version != 1 || c.X_density != 1 || c.Y_density != 1 ||
      *(int *)(c.comp_info + 0) != 1 || *(int *)(c.comp_info + COMP_INFO_SIZE) != 2 ||
      *(int *)(c.comp_info + 2 * COMP_INFO_SIZE) != 3 || *(int *)(c.comp_info + 8) != 2 ||
      *(int *)(c.comp_info + 12) != 2) {
    snprintf(g_why, sizeof g_why, "compress struct mirror does not match libjpeg's layout");
    g_state = -1;
    p_destroy(&c);
    free(buf);
    return 0;
  }
  p_set_quality(&c, quality, 1);
  c.dct_method = fastdct ? JDCT_IFAST : JDCT_ISLOW;
  p_set_colorspace(&c, subsamp == 3 ? JCS_GRAYSCALE : JCS_YCbCr);
  *(int *)(c.comp_info + 8) = samp_h[subsamp];
  *(int *)(c.comp_info + 12) = samp_v[subsamp];
  if (subsamp != 3)
    for (int k = 1; k < 3; ++k) {
      *(int *)(c.comp_info + k * COMP_INFO_SIZE + 8) = 1;
      *(int *)(c.comp_info + k * COMP_INFO_SIZE + 12) = 1;
    }
  c.restart_interval = (unsigned)restart_interval;
  c.restart_in_rows = restart_in_rows;
  c.optimize_coding = optimize;
  p_start_compress(&c, 1);
  while (c.next_scanline < (unsigned)h) {
    unsigned char *row = (unsigned char *)img + (size_t)c.next_scanline * w * 3;
    p_write_scanlines(&c, &row, 1);
  }
  p_finish_compress(&c);
  if (size <= cap) {
    memcpy(out, buf, size);
    result = size;
  }
  p_destroy(&c);
  free(buf);
  return result;
}

/* tjDecompress2(pixel_format BGR/RGB, flags) through libjpeg: w*h*3 bytes into `out`.
 * Returns 0 on success, -1 on failure. */
int xc_decode(const uint8_t *jpg, size_t n, int bgr, int fast_upsample, int w, int h, int ncomp,
              uint8_t *out) {
  static char dbuf[4096] __attribute__((aligned(16)));
  if (!xc_available(NULL, 0)) return -1;
  memset(dbuf, 0, sizeof dbuf);
  *(void **)dbuf = new_err();
  uint8_t *tmp = (uint8_t *)malloc((size_t)w * 3 + 16);
  if (!tmp) return -1;
  if (setjmp(g_jmp)) {
    p_destroy(dbuf);
    free(tmp);
    return -1;
  }
  p_CreateDecompress(dbuf, JPEG_LIB_VERSION, g_dsize);
  p_mem_src(dbuf, jpg, (unsigned long)n);
  p_read_header(dbuf, 1);
  if (*(unsigned *)(dbuf + D_IMAGE_WIDTH) != (unsigned)w || *(unsigned *)(dbuf + D_IMAGE_HEIGHT) != (unsigned)h ||
      *(int *)(dbuf + D_NUM_COMPONENTS) != ncomp ||
      *(int *)(dbuf + D_OUT_COLOR_SPACE) != (ncomp == 3 ? JCS_RGB : JCS_GRAYSCALE) ||
      *(unsigned *)(dbuf + D_SCALE_NUM) != 1 || *(unsigned *)(dbuf + D_SCALE_DENOM) != 1 ||
      *(int *)(dbuf + D_DCT_METHOD) != JDCT_ISLOW || *(int *)(dbuf + D_DO_FANCY_UPSAMPLING) != 1) {
    snprintf(g_why, sizeof g_why, "decompress struct offsets do not match libjpeg's layout");
    g_state = -1;
    p_destroy(dbuf);
    free(tmp);
    return -1;
  }
  if (ncomp == 3) *(int *)(dbuf + D_OUT_COLOR_SPACE) = bgr ? JCS_EXT_BGR : JCS_RGB;
  if (fast_upsample) *(int *)(dbuf + D_DO_FANCY_UPSAMPLING) = 0;
  p_start_decompress(dbuf);
  for (int y = 0; y < h; ++y) {
    unsigned char *row = tmp;
    if (p_read_scanlines(dbuf, &row, 1) != 1) {
      p_destroy(dbuf);
      free(tmp);
      return -1;
    }
    uint8_t *o = out + (size_t)y * w * 3;
    if (ncomp == 3) {
      memcpy(o, tmp, (size_t)w * 3);
    } else {
      for (int x = 0; x < w; ++x) o[3 * x] = o[3 * x + 1] = o[3 * x + 2] = tmp[x];
    }
  }
  p_finish_decompress(dbuf);
  p_destroy(dbuf);
  free(tmp);
  return 0;
}
