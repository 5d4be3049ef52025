// mpcx_internal.h -- kernel classes and launch arguments shared by the
// device code (mpcx_kernels.hip) and the C-ABI host code (mpcx_api.cpp).
#ifndef MPCX_INTERNAL_H_
#define MPCX_INTERNAL_H_

#include <stdint.h>

// A class serves odd moduli m of up to MPCX_CLASS_MAXBITS(c) bits; bases fit
// in MPCX_CLASS_WORDS(c) words. Each class is served by kernel geometries
// (P lanes per operand, K radix-2^28 digits per lane, G operands per 64-lane
// wavefront, L = P*K digits); every geometry of a class has R = 2^(28L) > 4m
// for the class's largest modulus, and its own Montgomery constants (R mod m,
// R^2 mod m depend on L), uploaded at registration.
#define MPCX_NUM_CLASSES 3
// class L_min: sets the class's operand width (every geometry of the class has
// L >= L_min digits; 147 is the round-1 7 x 21 geometry's, kept as the width)
#define MPCX_CLASS_LMIN(c) ((c) == 0 ? 37 : (c) == 1 ? 75 : 147)
// operand width in 32-bit words (bases and moduli)
#define MPCX_CLASS_WORDS(c) ((28 * MPCX_CLASS_LMIN(c)) / 32)
#define MPCX_CLASS_MAXBITS(c) (32 * MPCX_CLASS_WORDS(c))

// Geometries (id: P x K, G, class):
//   0: 1 x 37, 64, class 0  thread per operand (1024-bit safe-prime candidates, CRT halves)
//   1: 4 x 19, 16, class 1  quad per operand: m_i broadcast by DPP quad_perm (moduli of
//                           2071..2080 bits; fixed-base comb tables)
//   2: 4 x 37, 16, class 2  quad per operand (Paillier N^2)
//   3: 16 x 5,  4, class 1  narrow: small latency-bound batches; one DPP row per operand,
//                           m_i broadcast by DPP row_newbcast
//   4: 32 x 5,  2, class 2  narrow; two DPP rows per operand, m_i by row_newbcast + row_bcast:15
//   5: 2 x 37, 32, class 1  lane pair per operand, m_i by DPP quad_perm [0,0,2,2]: the 2048-bit
//                           main geometry (N, N~). L = 74 < the class's L_min: R = 2^2072 > 4m
//                           needs m < 2^2070 and operands < 2^2072 (MPCX_GEOM_RBITS), checked
//                           per launch; otherwise geometry 1 serves the launch
//   6: 8 x 19,  8, class 2  mid: batches of a fraction of a main round (twice the main
//                           geometry's wavefronts, 3 per SIMD); m_i by quad_perm + row_shr:4
#define MPCX_NUM_GEOMS 7
#define MPCX_GEOM_P(g) \
  ((g) == 0 ? 1 : (g) == 1 ? 4 : (g) == 2 ? 4 : (g) == 3 ? 16 : (g) == 4 ? 32 : (g) == 5 ? 2 : 8)
#define MPCX_GEOM_K(g) \
  ((g) == 0 ? 37 : (g) == 1 ? 19 : (g) == 2 ? 37 : (g) == 3 ? 5 : (g) == 4 ? 5 : (g) == 5 ? 37 : 19)
#define MPCX_GEOM_G(g) \
  ((g) == 0 ? 64 : (g) == 1 ? 16 : (g) == 2 ? 16 : (g) == 3 ? 4 : (g) == 4 ? 2 : (g) == 5 ? 32 : 8)
#define MPCX_GEOM_CLASS(g) ((g) == 0 ? 0 : ((g) == 1 || (g) == 3 || (g) == 5) ? 1 : 2)
#define MPCX_GEOM_L(g) (MPCX_GEOM_P(g) * MPCX_GEOM_K(g))
// bits of R = 2^(28 L): a geometry serves moduli m with 4m < R and operands below R
#define MPCX_GEOM_RBITS(g) (28 * MPCX_GEOM_L(g))
// default main (throughput) and narrow geometry of each class
#define MPCX_MAIN_GEOM(c) ((c) == 0 ? 0 : (c) == 1 ? 5 : 2)
#define MPCX_NARROW_GEOM(c) ((c) == 1 ? 3 : (c) == 2 ? 4 : -1)
#define MPCX_MID_GEOM(c) ((c) == 2 ? 6 : -1)
// the geometry every modulus of the class can use (L >= L_min), and the layout of
// the class's fixed-base comb tables
#define MPCX_FULL_GEOM(c) ((c) == 0 ? 0 : (c) == 1 ? 1 : 2)
// 1024-bit class used by the Fermat / Miller-Rabin kernels (thread per operand)
#define MPCX_C0_K 37

// table entries per wavefront in the workspace: powers p_0..p_15 (fixed
// window) or the odd powers x, x^3, ..., x^63 (sliding window, table[0..31]),
// + the Montgomery form of the optional multiplier (entry 32)
#define MPCX_TABLE_ENTRIES 34
#define MPCX_MUL_ENTRY 32
// k_modexp_mx: x^2 R, the odd-power chain's multiplier, staged again before each
// product (montmul_mx overwrites its LDS row)
#define MPCX_SQ_ENTRY 33

// Sliding-window schedule of a shared exponent (built by k_expsched on the
// launch stream, read by k_modexp through scalar loads):
//   [TOP]   odd-power table index of the top window (x^(2 top + 1)),
//           MPCX_SCHED_NONE for e = 0
//   [TN]    highest odd-power index used (table[0..TN] = x^1, x^3, ...)
//   [N]     number of steps
//   [WIDTH] window width (bits) the schedule was built with
//   [STEPS + i]  (squarings << 8) | odd-power index (0xFF: squarings only)
#define MPCX_SCHED_TOP 0
#define MPCX_SCHED_TN 1
#define MPCX_SCHED_N 2
#define MPCX_SCHED_WIDTH 3
#define MPCX_SCHED_STEPS 4
#define MPCX_SCHED_NONE 0xFFFFFFFFu
#define MPCX_SCHED_MAX_WIDTH 6  // 2^(w-1) <= 32 odd powers fit table[0..31]
// schedule words for an exponent of `bits` bits (at most one step per bit)
#define MPCX_SCHED_WORDS(bits) (MPCX_SCHED_STEPS + (bits) + 1)

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
  uint32_t exp_bits;    // fixed window: windows processed = ceil(exp_bits / win_bits)
  uint32_t win_bits;    // fixed-window width (4 or 5): table p_0..p_(2^win_bits - 1)
  uint32_t out_words;
  uint32_t n0inv;       // -m^-1 mod 2^28
  int exp_shared;
  const uint32_t* sched; // shared exponent: its window schedule (nullptr: fixed window)
  // geometry 2 only: the LDS image of the Toeplitz tables of m'' = -m^-1 mod R and
  // of m (mpcx_mx.hpp, 2 x MPCX_MX_TAB_BYTES): k_modexp_mx, the reduction on the
  // matrix cores, MX_WG wavefronts per workgroup. nullptr: k_modexp
  const void* mx_img;
  uint32_t nwaves;      // wavefronts with work (k_modexp_mx: the last workgroup's spare waves exit)
};
// workgroup: MX_WG wavefronts share the Toeplitz tables and m's digits in LDS
#ifndef MX_WG
#define MX_WG 4
#endif

// An MX geometry: P lanes x K radix-2^28 digits per operand, G operands per wave.
template <int P_, int K_, int G_>
struct MxShape {
  static constexpr int P = P_, K = K_, G = G_, L = P * K;
  static constexpr int HALVES = G / 16;  // 16 operands per MFMA column set
  static constexpr int N7 = 4 * L;       // radix-2^7 digits of R
  // dwords per operand row: 16-B aligned, an odd number of 16-B slots (ds_read_b128
  // of 16 rows conflict-free)
  static constexpr int ROW = (((L + 3) / 4) % 2 == 1 ? (L + 3) / 4 : (L + 3) / 4 + 1) * 4;
  static constexpr int KB = (N7 + 63) / 64;          // K blocks of 64 digits
  static constexpr int O1 = (N7 + 15) / 16;          // output blocks of q (digits >= L zeroed)
  static constexpr int NJ1 = O1;                     // Toeplitz blocks of m'' (delta = 16 j)
  static constexpr int NJ2 = (N7 + 62) / 16 + 1;     // Toeplitz blocks of m with a non-zero entry
  static constexpr int JMAX = (NJ1 > NJ2 ? NJ1 : NJ2) - 1;
  static constexpr int D = 16 * JMAX;                // table copy_i[x] = v7[D - x + i]
  static constexpr int TAB_STRIDE = (((D + 64) / 16) % 2 == 1 ? (D + 64) / 16 : (D + 64) / 16 + 1) * 16;
  static constexpr int TAB_BYTES = 16 * TAB_STRIDE;
  static constexpr int IMG_BYTES = 2 * TAB_BYTES;    // the LDS image of both tables (the C-ABI uploads it)
  static constexpr int O2LO = (N7 - 4) / 16;         // block of the low half's top 4 positions (the carry)
  static constexpr int O2HI = (2 * N7 + 15) / 16;    // one past U's top block
#ifndef MX_CS
#define MX_CS 13
#endif
  static constexpr int CS1 = MX_CS, CS2 = MX_CS;     // output blocks per chunk (live accumulators)
  // +4: the product loop reads one past the last row; then the product loop's
  // trash slots (lanes p != 0 store there: lane + digit index < 64 + L)
  static constexpr int TRASH_OFF = G * ROW + 4;
  static constexpr int WAVE_WORDS = TRASH_OFF + ((64 + L + 3) / 4) * 4;
  static constexpr int LDS_WORDS_WG = IMG_BYTES / 4 + L + 4 + MX_WG * WAVE_WORDS;
};
// k_modexp_mx geometries (mpcx_mx.hpp)
using MxG2 = MxShape<4, 37, 16>;  // geometry 2: R = 2^4144, 592 radix-2^7 digits
using MxG5 = MxShape<2, 37, 32>;  // geometry 5: R = 2^2072, 296 radix-2^7 digits


// Fixed-base tables (mpcx_fixedbase_register): w-bit windows (w chosen per
// table, <= MPCX_FB_MAX_WINDOW_BITS); for window j < nwin and value v < 2^w,
// entry (j, v) = b^(v * 2^(w j)) R mod m as L radix-2^28 digits of the class's
// main geometry, interleaved [digit slot k][lane p] so a group's P lanes read
// P consecutive words per slot. Entry (j, 0) = R mod m.
#define MPCX_FB_WINDOW_BITS 12      // default width (option "fb_window")
#define MPCX_FB_MAX_WINDOW_BITS 12
#define MPCX_FB_MAX_TABLE_BYTES (512ull << 20)  // narrower windows above this per table
// most wavefronts one comb operand's windows are split over (k_fixedbase)
#define MPCX_FB_MAX_SPLIT 4
#ifndef MPCX_FB_MAX_BASES
#define MPCX_FB_MAX_BASES 2  // also in include/mpcx.h
#endif

struct FixedBaseArgs {
  const uint32_t* nd;   // L digits of m
  const uint32_t* r1d;  // L digits of R mod m (Montgomery one)
  const uint32_t* r2d;  // L digits of R^2 mod m
  const uint32_t* tables[MPCX_FB_MAX_BASES];
  const uint32_t* exps[MPCX_FB_MAX_BASES];  // count x exp_words[t]
  uint32_t exp_words[MPCX_FB_MAX_BASES];
  uint32_t nwin[MPCX_FB_MAX_BASES];         // windows processed per base
  uint32_t wbits[MPCX_FB_MAX_BASES];        // window width of each base's table
  uint32_t nbases;
  const uint32_t* mul;  // optional count x mul_words multipliers
  uint32_t mul_words;
  uint32_t* out;        // count x out_words
  uint32_t out_words;
  uint32_t count;
  uint32_t n0inv;
};

struct ExpSchedArgs {
  const uint32_t* exp;  // shared exponent, exp_words little-endian words
  uint32_t exp_words;
  uint32_t max_width;   // cap on the window width (1..MPCX_SCHED_MAX_WIDTH)
  uint32_t* sched;      // MPCX_SCHED_WORDS(32 * exp_words) words
};


// Safe-prime candidate sieve (tss-lib runGenPrimeRoutine steps 1-3 plus exact
// trial division of q and 2q+1, up:common/safe_prime.go): one thread per
// candidate; survivors p = 2q+1 are appended (atomic slot) with their index.
#define MPCX_SIEVE_MAX_BYTES 128  // q of <= 1023 bits
struct SieveArgs {
  const uint8_t* raw;        // count x nbytes big-endian random bytes (the stream)
  uint32_t nbytes, count, q_bits;
  const uint32_t* tprod;     // trial groups: product of primes (< 2^32)
  const uint64_t* tinv;      // floor((2^64 - 1) / tprod)
  const uint32_t* tstart;    // group g's primes: tprimes[tstart[g] .. tstart[g+1])
  const uint32_t* tprimes;
  uint32_t ngroups;
  uint32_t* out_p;           // survivors: count x 32 words (p = 2q + 1)
  uint32_t* out_idx;         // survivors' candidate indices
  uint32_t* out_count;       // survivor counter (zeroed before the launch)
};

// Base-2 tests of the safe-prime search (k_prime2), one candidate per lane:
// blocks [0, f_blocks): Fermat items 2^(n-1) == 1 (mod n) over the sieve
// survivors nf[0 .. min(count_f, *count_dev)); blocks [f_blocks, ...): strong
// probable-prime-to-base-2 items over ns[0 .. count_s) (the Fermat passes' q
// of an earlier batch riding along in the same launch). n: n_words words.
struct Prime2Args {
  const uint32_t* nf;
  uint32_t count_f;
  const uint32_t* count_dev;  // optional: Fermat items = min(count_f, *count_dev)
  uint32_t f_blocks;
  uint8_t* ok_f;              // optional: per-item Fermat verdicts
  // optional compaction of the Fermat passes: slot = atomicAdd(pass_count, 1),
  // pass_idx[slot] = sieve_idx[item], pass_n[slot] = the item's n_words words
  const uint32_t* sieve_idx;
  uint32_t* pass_count;
  uint32_t* pass_idx;
  uint32_t* pass_n;
  const uint32_t* ns;
  uint32_t count_s;
  uint8_t* ok_s;
  uint32_t n_words;
  // cooperative kernels (k_pprep_prime2 + k_prime2c): per-item constants for
  // the Fermat items [0, count_f) then the strong items (offset count_f)
  uint32_t* r1;        // (count_f + count_s) x MPCX_PRIME_L digits: R mod n
  uint32_t* meta;      // (count_f + count_s) x 2: -n^-1 mod 2^28, nbits | s << 16
  uint32_t fp_blocks;  // prep blocks (64 items) of the Fermat segment
};

// Cooperative per-candidate geometries (P lanes x K digits per candidate,
// L = P K digits, R = 2^(28 L) > 16 n for n < 2^1024): the base-2 tests of
// the safe-prime step, and Miller-Rabin with arbitrary bases (latency-bound
// batches: 16 lanes per test).
#define MPCX_PRIME_P 2
#define MPCX_PRIME_K 19
#define MPCX_PRIME_L (MPCX_PRIME_P * MPCX_PRIME_K)
#define MPCX_MR_P 16
#define MPCX_MR_K 3
#define MPCX_MR_L (MPCX_MR_P * MPCX_MR_K)
// the strong Lucas test of wider candidates (2^1024 <= n < 2^2048: ModProof's
// N.ProbablyPrime): 16 lanes x 5 digits, R = 2^(28 * 80) > 16 n
#define MPCX_LUCASW_K 5
#define MPCX_LUCASW_L (MPCX_MR_P * MPCX_LUCASW_K)

// Strong Lucas probable-prime test (Go math/big probablyPrimeLucas, the
// "extra strong" test with Baillie-OEIS method C parameters P, Q = 1,
// D = P^2 - 4 with Jacobi(D, n) = -1; P is chosen by the caller).
struct LucasArgs {
  const uint32_t* n;   // count x n_words odd candidates, 5 <= n < 2^1024
  const uint32_t* P;   // count parameters (3 <= P < 2^14)
  uint8_t* ok;
  uint32_t count;
  uint32_t n_words;
  // cooperative kernel (k_pprep_lucas + k_lucasc, MPCX_MR_L digits): per item
  // P R, 2 R, 2n - P R, 2n - 2 R (Montgomery forms) and n0inv, nbits | r << 16
  uint32_t* consts;  // count x 4 x MPCX_MR_L digits
  uint32_t* meta;    // count x 2
};

// The build's CounterDRBG stream on the device: block c (32 bytes) =
// SHA-256("mpcx-drbg" || seed as 8 LE bytes || c as 8 LE bytes); out[i] =
// stream byte off + i for i < n.
struct DrbgArgs {
  uint64_t seed;
  uint64_t off;
  uint64_t n;
  uint8_t* out;
};

struct MrArgs {
  const uint32_t* n;  // count x n_words odd candidates
  const uint32_t* a;  // count x n_words bases (< 2^(32*n_words))
  uint8_t* ok;
  uint32_t count;
  uint32_t n_words;
  uint32_t* r1;    // cooperative kernel: count x MPCX_MR_L digits (k_pprep_mr)
  uint32_t* meta;  // count x 2
};

}  // namespace mpcx

#endif
