// pnm.h -- gray/colour PNM I/O of the reference API (drop-in for /root/reference/src/pnm.h).
// tipo = the digit of the magic number (2 = ASCII gray, 5 = binary gray, 6 = binary RGB);
// ancho = width, alto = height. Samples are pixel_t; P5 with maxval >= 256 is 16-bit big-endian.
#ifndef PNM_H
#define PNM_H

#include <cstdio>

typedef unsigned int pixel_t;

// Returns 0, or -1 on a bad magic number (the file is then closed, as in pnm.cpp:23-31) or a
// missing field. Comment lines are allowed before each of the three numbers.
int read_pnm_header(FILE* f, int& tipo, int& ancho, int& alto, int& maxval);
// Reads ancho*alto samples; for P5 returns the number of samples missing (0 = complete).
int read_pgm_data(FILE* f, int tipo, int ancho, int alto, int maxval, pixel_t* buf);
int read_ppm_data(FILE* f, int tipo, int ancho, int alto, int maxval, pixel_t* buf);

int write_pgm(const pixel_t* pixels, int tipo, int ancho, int alto, int maxval, const char* ruta_archivo);
int write_ppm(const pixel_t* pixels, int tipo, int ancho, int alto, int maxval, const char* ruta_archivo);
int write_ppm_header(int tipo, int ancho, int alto, int maxval, FILE* ruta_archivo);
int write_p2_data(const pixel_t* pixels, const int npixels, const int maxval, FILE* fw);
int write_p5_data(const pixel_t* pixels, const int npixels, const int maxval, FILE* fw);

#endif
