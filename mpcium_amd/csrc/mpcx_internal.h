// mpcx_internal.h -- kernel classes and launch arguments shared by the
// device code (mpcx_kernels.hip) and the C-ABI host code (mpcx_api.cpp).
#ifndef MPCX_INTERNAL_H_
#define MPCX_INTERNAL_H_

#include <stdint.h>

// A class serves odd moduli m with R = 2^(28L) > 4m and bases that fit in
// floor(28L/32) words:
//   P: lanes per operand, K: radix-2^28 digits per lane, G: operands per
//   64-lane wavefront (G*P <= 64), L = P*K digits.
#define MPCX_NUM_CLASSES 3
// class 0: moduli up to 1024 bits (1024-bit safe-prime candidates p)
#define MPCX_C0_P 1
#define MPCX_C0_K 37
#define MPCX_C0_G 64
// class 1: moduli up to 2080 bits (Paillier N, N~)
#define MPCX_C1_P 3
#define MPCX_C1_K 25
#define MPCX_C1_G 21
// class 2: moduli up to 4096 bits (Paillier N^2)
#define MPCX_C2_P 7
#define MPCX_C2_K 21
#define MPCX_C2_G 9

#define MPCX_CLASS_P(c) ((c) == 0 ? MPCX_C0_P : (c) == 1 ? MPCX_C1_P : MPCX_C2_P)
#define MPCX_CLASS_K(c) ((c) == 0 ? MPCX_C0_K : (c) == 1 ? MPCX_C1_K : MPCX_C2_K)
#define MPCX_CLASS_G(c) ((c) == 0 ? MPCX_C0_G : (c) == 1 ? MPCX_C1_G : MPCX_C2_G)
#define MPCX_CLASS_L(c) (MPCX_CLASS_P(c) * MPCX_CLASS_K(c))
// Kernel geometries. Geometry c < MPCX_NUM_CLASSES is class c's main
// (throughput) geometry; the "narrow" ones split the same L digits over more
// lanes (fewer digits per lane -> ~3x shorter wavefronts) and serve the last
// partial round of a batch and small, latency-bound batches.
#define MPCX_NUM_GEOMS 5
#define MPCX_G3_P 15  // class 1 narrow: 15 x 5 = 75 digits, 4 operands per wave
#define MPCX_G3_K 5
#define MPCX_G3_G 4
#define MPCX_G4_P 21  // class 2 narrow: 21 x 7 = 147 digits, 3 operands per wave
#define MPCX_G4_K 7
#define MPCX_G4_G 3
#define MPCX_GEOM_P(g) ((g) < 3 ? MPCX_CLASS_P(g) : (g) == 3 ? MPCX_G3_P : MPCX_G4_P)
#define MPCX_GEOM_K(g) ((g) < 3 ? MPCX_CLASS_K(g) : (g) == 3 ? MPCX_G3_K : MPCX_G4_K)
#define MPCX_GEOM_G(g) ((g) < 3 ? MPCX_CLASS_G(g) : (g) == 3 ? MPCX_G3_G : MPCX_G4_G)
#define MPCX_NARROW_GEOM(c) ((c) == 1 ? 3 : (c) == 2 ? 4 : -1)

// operand width in 32-bit words (bases and moduli)
#define MPCX_CLASS_WORDS(c) ((28 * MPCX_CLASS_L(c)) / 32)
#define MPCX_CLASS_MAXBITS(c) (32 * MPCX_CLASS_WORDS(c))

// table entries per wavefront in the workspace: powers p_0..p_15 + the
// Montgomery form of the optional multiplier (entry 16)
#define MPCX_TABLE_ENTRIES 17

namespace mpcx {

struct ModexpArgs {
  const uint32_t* nd;   // L digits of m (radix 2^28)
  const uint32_t* r1d;  // L digits of R mod m
  const uint32_t* r2d;  // L digits of R^2 mod m
  const uint32_t* base; // count x base_words
  const uint32_t* exps; // 1 or count x exp_words
  const uint32_t* mul;  // optional count x mul_words multipliers (nullptr: none)
  uint32_t* out;        // count x out_words
  uint32_t* table;      // workspace: waves x MPCX_TABLE_ENTRIES x K x 64 words
  uint32_t count;
  uint32_t base_words;
  uint32_t exp_words;
  uint32_t mul_words;
  uint32_t exp_bits;    // windows processed = ceil(exp_bits / 4)
  uint32_t out_words;
  uint32_t n0inv;       // -m^-1 mod 2^28
  int exp_shared;
};

struct FermatArgs {
  const uint32_t* p;  // count x p_words candidates
  uint8_t* ok;
  uint32_t count;
  uint32_t p_words;
};

struct MrArgs {
  const uint32_t* n;  // count x n_words odd candidates
  const uint32_t* a;  // count x n_words bases (< 2^(32*n_words))
  uint8_t* ok;
  uint32_t count;
  uint32_t n_words;
};

}  // namespace mpcx

#endif
