// eg.h -- block run-length ("EG") coder of the reference API (drop-in for
// /root/reference/src/eg.h). State: g = log2(block size), blockSize, lutIndex into the JPEG-LS
// run-index table. As in the reference, the block size never grows (codeRun does not call
// incBlockSize, eg.cpp:25), so a run of length len costs len + 1 bits, and the first non-EOL run
// one bit more (g = 1 until then, 0 after).
#ifndef EG_H
#define EG_H

namespace bic {
struct coder_state;
}

class EG {
 public:
  EG() : g(1), blockSize(1), lutIndex(0) {}
  unsigned g;
  unsigned blockSize;
  int lutIndex;
  void incBlockSize();
  void decBlockSize();
};

class EGCoder : public EG {
 public:
  EGCoder() : EG(), bitcount() {}
  void codeRun(int len, bool eol);
  unsigned long bitcount;
};

// Declared by the reference, whose decoder body is disabled (eg.cpp:41-55); the stream decoder
// of this build is bic::EGStreamDecoder in bic_gpu.h.
class EGDecoder : public EG {
 public:
  EGDecoder() : EG() {}
  int decodeRun(int maxlen);
};

#endif
