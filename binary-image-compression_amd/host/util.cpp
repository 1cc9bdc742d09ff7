// util.cpp -- include/util.h, after /root/reference/src/util.cpp:4-90.
#include "util.h"

#include <cmath>
#include <vector>

#include "pbm.h"

void counting_sort(aux_t* s, idx_t n) {
  idx_t top = 0;
  for (idx_t i = 0; i < n; ++i) top = s[i].first > top ? s[i].first : top;
  // start[v] = number of keys < v. As in util.cpp:34-43 the elements are dealt from the
  // back of the input into increasing slots, so equal keys come out in REVERSE input order, and
  // both fields pass through int.
  std::vector<idx_t> start(top + 2, 0);
  for (idx_t i = 0; i < n; ++i) ++start[s[i].first + 1];
  for (idx_t v = 1; v <= top + 1; ++v) start[v] += start[v - 1];
  std::vector<aux_t> out(n);
  for (idx_t i = n; i-- > 0;) {
    const int key = (int)s[i].first, val = (int)s[i].second;
    out[start[key]++] = aux_t((idx_t)(long)key, (idx_t)(long)val);
  }
  for (idx_t i = 0; i < n; ++i) s[i] = out[i];
}

// Row li of D is a vectorised w x w patch, w = floor(sqrt(cols)); patches go on a grid of
// gn columns and ceil(rows/gn) rows with a one-pixel gutter (util.cpp:53-82).
void render_mosaic(const binary_matrix& D, const char* fname) {
  const idx_t m = D.get_cols();
  const idx_t n = D.get_rows();
  const idx_t w = (idx_t)std::sqrt(double(m));
  const idx_t gn = (idx_t)std::ceil(std::sqrt(double(n)));
  const idx_t gm = (idx_t)std::ceil(double(n) / double(gn));
  const idx_t gw = w + 1;
  binary_matrix I(gm * gw, gn * gw);
  binary_matrix V(1, m);
  binary_matrix P(w, w);
  I.clear();
  for (idx_t li = 0; li < n; ++li) {
    D.copy_row_to(li, V);
    P.set_vectorized(V);
    I.set_submatrix(gw * (li / gn), gw * (li % gn), P);
  }
  FILE* f = fopen(fname, "w");
  if (f) {
    write_pbm(I, f);
    fclose(f);
  }
  I.destroy();
  V.destroy();
  P.destroy();
}

int write_pbm(binary_matrix& A, const char* fname) {
  FILE* f = fopen(fname, "w");
  if (!f) return -2;
  write_pbm(A, f);
  fclose(f);
  return 0;
}
