// pnm.cpp -- PNM I/O (include/pnm.h) with the observable behaviour of
// /root/reference/src/pnm.cpp:5-239: same fields consumed, same return values, same samples in
// `buf` (including what a short 16-bit raster leaves behind). Rasters are read in bulk.
#include "pnm.h"

#include <cctype>
#include <vector>

namespace {

// Skips whitespace and '#' comment lines, leaving the stream on the next other character
// (pnm.cpp:5-18; a comment is consumed 99 characters at a time, like its fgets buffer).
void skip_comments(FILE* fp) {
  for (;;) {
    int ch;
    while ((ch = fgetc(fp)) != EOF && isspace(ch)) {
    }
    if (ch != '#') {
      fseek(fp, -1, SEEK_CUR);
      return;
    }
    char line[100];
    if (!fgets(line, sizeof(line), fp)) {
      fseek(fp, -1, SEEK_CUR);  // what the reference's recursion does at end of file
      return;
    }
  }
}

int read_p2(FILE* f, int ancho, int alto, pixel_t* buf) {
  const int n = ancho * alto;
  for (int i = 0; i < n; ++i)
    if (fscanf(f, "%u", &buf[i]) <= 0) break;
  return 0;
}

int read_p5(FILE* f, int ancho, int alto, int maxval, pixel_t* buf) {
  const int n = ancho * alto;
  int got;
  if (maxval < 256) {
    std::vector<unsigned char> raw(n > 0 ? n : 0);
    got = n > 0 ? (int)fread(raw.data(), 1, n, f) : 0;
    for (int i = 0; i < got; ++i) buf[i] = raw[i];
  } else {
    std::vector<unsigned char> raw(n > 0 ? 2 * (size_t)n : 0);
    const size_t bytes = n > 0 ? fread(raw.data(), 1, 2 * (size_t)n, f) : 0;
    got = (int)(bytes / 2);
    for (int i = 0; i < got; ++i) buf[i] = ((pixel_t)raw[2 * i] << 8) | raw[2 * i + 1];
    // after a short read the reference keeps assigning from its 2-byte buffer, which holds the
    // last bytes that did arrive (an odd trailing byte replaces only the high byte)
    if (got < n) {
      unsigned char hi = got ? raw[2 * got - 2] : 0, lo = got ? raw[2 * got - 1] : 0;
      if (bytes & 1) hi = raw[bytes - 1];
      for (int i = got; i < n; ++i) buf[i] = ((pixel_t)hi << 8) | lo;
    }
  }
  if (got < n)
    printf("Only %d samples read, %d expected: feof()=%d\tferror()=%d\n", got, n, feof(f), ferror(f));
  return n - got;
}

int write_gray(const pixel_t* pixels, int tipo, int ancho, int alto, int maxval, const char* path) {
  FILE* fw = fopen(path, "wb");
  if (!fw) {
    printf("Cannot write %s\n", path);
    return -1;
  }
  write_ppm_header(tipo, ancho, alto, maxval, fw);
  if (tipo == 2)
    write_p2_data(pixels, ancho * alto, maxval, fw);
  else
    write_p5_data(pixels, ancho * alto, maxval, fw);
  return fclose(fw);
}

}  // namespace

int read_pnm_header(FILE* f, int& tipo, int& ancho, int& alto, int& maxval) {
  if (fgetc(f) != 'P') {
    printf("Not a PNM file.\n");
    fclose(f);
    return -1;
  }
  tipo = fgetc(f) - '0';
  if (tipo != 2 && tipo != 5 && tipo != 6) {
    printf("Unsupported PNM type %d (2, 5 or 6 expected)\n", tipo);
    fclose(f);
    return -1;
  }
  int* fields[3] = {&ancho, &alto, &maxval};
  for (int* v : fields) {
    skip_comments(f);
    if (fscanf(f, "%d", v) <= 0) return -1;
  }
  fgetc(f);  // the single whitespace byte before the raster
  return 0;
}

int read_pgm_data(FILE* f, int tipo, int ancho, int alto, int maxval, pixel_t* buf) {
  if (tipo == 2) return read_p2(f, ancho, alto, buf);
  if (tipo == 5) return read_p5(f, ancho, alto, maxval, buf);
  return 0;
}

int read_ppm_data(FILE* f, int, int ancho, int alto, int, pixel_t* buf) {
  const int n = ancho * alto;
  std::vector<unsigned char> rgb(n > 0 ? 3 * (size_t)n : 0);
  const size_t bytes = n > 0 ? fread(rgb.data(), 1, rgb.size(), f) : 0;
  const int got = (int)(bytes / 3);
  for (int i = 0; i < got; ++i)
    buf[i] = ((pixel_t)rgb[3 * i] << 16) | ((pixel_t)rgb[3 * i + 1] << 8) | rgb[3 * i + 2];
  if (got < n) {
    // the reference stores the pixel whose read failed, then stops (pnm.cpp:199-208)
    unsigned char c[3] = {got ? rgb[3 * got - 3] : (unsigned char)0, got ? rgb[3 * got - 2] : (unsigned char)0,
                          got ? rgb[3 * got - 1] : (unsigned char)0};
    for (size_t b = 3 * (size_t)got; b < bytes; ++b) c[b - 3 * (size_t)got] = rgb[b];
    buf[got] = ((pixel_t)c[0] << 16) | ((pixel_t)c[1] << 8) | c[2];
    return got + 1 < n ? -1 : 0;  // its loop counter has already passed the failed pixel
  }
  return 0;
}

int write_ppm_header(int tipo, int ancho, int alto, int maxval, FILE* fw) {
  fprintf(fw, "P%c\n", tipo + '0');
  fprintf(fw, "%d %d\n", ancho, alto);
  fprintf(fw, "%d\n", maxval);
  return ferror(fw);
}

int write_p2_data(const pixel_t* pixels, const int npixels, const int, FILE* fw) {
  for (int i = 0; i < npixels; ++i) {
    fprintf(fw, "%d\t", pixels[i]);
    if ((i + 1) % 20 == 0) fprintf(fw, "\n");
  }
  return ferror(fw);
}

int write_p5_data(const pixel_t* pixels, const int npixels, const int maxval, FILE* fw) {
  const int width = maxval < 256 ? 1 : 2;
  std::vector<unsigned char> raw(npixels > 0 ? (size_t)npixels * width : 0);
  for (int i = 0; i < npixels; ++i) {
    if (width == 1) {
      raw[i] = (unsigned char)pixels[i];
    } else {
      raw[2 * i] = (unsigned char)(pixels[i] >> 8);
      raw[2 * i + 1] = (unsigned char)pixels[i];
    }
  }
  if (!raw.empty()) fwrite(raw.data(), 1, raw.size(), fw);
  return ferror(fw);
}

int write_pgm(const pixel_t* pixels, int tipo, int ancho, int alto, int maxval, const char* path) {
  if (tipo != 2 && tipo != 5) return -1;
  return write_gray(pixels, tipo, ancho, alto, maxval, path);
}

int write_ppm(const pixel_t* pixels, int, int ancho, int alto, int maxval, const char* path) {
  FILE* f = fopen(path, "wb");
  if (!f) {
    printf("Cannot write %s\n", path);
    return -1;
  }
  fprintf(f, "P6\n%d %d\n%d\n", ancho, alto, maxval);
  const int n = ancho * alto;
  std::vector<unsigned char> rgb(n > 0 ? 3 * (size_t)n : 0);
  for (int i = 0; i < n; ++i) {
    rgb[3 * i] = (unsigned char)(pixels[i] >> 16);
    rgb[3 * i + 1] = (unsigned char)(pixels[i] >> 8);
    rgb[3 * i + 2] = (unsigned char)pixels[i];
  }
  if (!rgb.empty()) fwrite(rgb.data(), 1, rgb.size(), f);
  fclose(f);
  return 0;
}
