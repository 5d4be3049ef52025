/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this file's build product (oracle/libgomodexp.so). The product path
 * (mpcium_amd/, libmpcx.so) never links, loads or calls it.
 *
 * Plain-C restatement of Go math/big modular exponentiation as the reference
 * reaches it: tss-lib v2.0.2 common.ModInt(m).Exp(x, y) = new(big.Int).Exp(x, y, m)
 * (up:common/int.go, pinned by /root/reference/go.mod:10), toolchain go1.23.5
 * (/root/reference/go.mod:5). Restated functions:
 *   (*Int).Exp / (*Int).exp        go:src/math/big/int.go    -> go_int_exp()
 *   nat.expNN                      go:src/math/big/nat.go    -> nat_expNN()
 *   nat.expNNMontgomery            go:src/math/big/nat.go    -> nat_expNNMontgomery()
 *   nat.montgomery (AMM, Gueron)   go:src/math/big/nat.go    -> nat_montgomery()
 * Word size: built twice by oracle/Makefile. libgomodexp.so uses 32-bit words
 * (the parity oracle of the tests); libgomodexp64.so (-DGOMODEXP_W64) uses
 * 64-bit Words with 128-bit products, Go's amd64 configuration (_W = 64,
 * arith_amd64.s addMulVVW = MULQ/ADC chains), and is the CPU baseline of
 * bench.py. The word size changes the number of Montgomery steps per word but
 * not the integer result (x^y mod m is unique). The single-word-exponent
 * square-and-multiply branch of expNN is taken, as on amd64, when y < 2^64.
 *
 * Parity status: the reference (Go + tss-lib) cannot be built or run in this
 * image (no Go toolchain, tss-lib absent). This restatement is
 * pinned instead against three independent bignum implementations (CPython
 * pow, GMP mpz_powm, OpenSSL BN_mod_exp) through tests/golden/ -- "parity
 * unpinned" with respect to the reference's own fixtures, which do not exist.
 *
 * Build: make -C oracle   (gcc only, no dependencies)
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef GOMODEXP_W64
typedef uint64_t Word;
typedef unsigned __int128 DWord;
typedef __int128 SDWord;
#define WBITS 64
#define CLZ(x) __builtin_clzll(x)
#define EXPORT static __attribute__((unused))
#else
typedef uint32_t Word;
typedef uint64_t DWord;
typedef int64_t SDWord;
#define WBITS 32
#define CLZ(x) __builtin_clz(x)
#define EXPORT
#endif

/* ---------- nat helpers (go:src/math/big/arith.go, nat.go) ---------- */

static int nat_norm(const Word* x, int n) {
  while (n > 0 && x[n - 1] == 0) n--;
  return n;
}

static int nat_cmp(const Word* x, int nx, const Word* y, int ny) {
  nx = nat_norm(x, nx);
  ny = nat_norm(y, ny);
  if (nx != ny) return nx < ny ? -1 : 1;
  for (int i = nx - 1; i >= 0; i--) {
    if (x[i] != y[i]) return x[i] < y[i] ? -1 : 1;
  }
  return 0;
}

/* z = x - y (n words), returns borrow. arith.go subVV */
static Word subVV(Word* z, const Word* x, const Word* y, int n) {
  Word c = 0;
  for (int i = 0; i < n; i++) {
    DWord d = (DWord)x[i] - y[i] - c;
    z[i] = (Word)d;
    c = (Word)((d >> (2 * WBITS - 1)) & 1);
  }
  return c;
}

/* z += x*y (n words), returns carry. arith.go addMulVVW */
static Word addMulVVW(Word* z, const Word* x, Word y, int n) {
  Word c = 0;
  for (int i = 0; i < n; i++) {
    DWord t = (DWord)x[i] * y + z[i] + c;
    z[i] = (Word)t;
    c = (Word)(t >> WBITS);
  }
  return c;
}

/* Knuth algorithm D: r = u mod v (q discarded). Writes r (nv words). nat.go div/divLarge. */
static void nat_rem(Word* r, const Word* u_in, int nu, const Word* v_in, int nv) {
  nu = nat_norm(u_in, nu);
  nv = nat_norm(v_in, nv);
  memset(r, 0, sizeof(Word) * nv);
  if (nat_cmp(u_in, nu, v_in, nv) < 0) {
    memcpy(r, u_in, sizeof(Word) * nu);
    return;
  }
  if (nv == 1) {
    DWord rem = 0;
    for (int i = nu - 1; i >= 0; i--) rem = ((rem << WBITS) | u_in[i]) % v_in[0];
    r[0] = (Word)rem;
    return;
  }
  int s = CLZ(v_in[nv - 1]);
  Word* v = (Word*)calloc(nv, sizeof(Word));
  Word* u = (Word*)calloc(nu + 1, sizeof(Word));
  for (int i = nv - 1; i > 0; i--) v[i] = s ? (v_in[i] << s) | (v_in[i - 1] >> (WBITS - s)) : v_in[i];
  v[0] = v_in[0] << s;
  u[nu] = s ? u_in[nu - 1] >> (WBITS - s) : 0;
  for (int i = nu - 1; i > 0; i--) u[i] = s ? (u_in[i] << s) | (u_in[i - 1] >> (WBITS - s)) : u_in[i];
  u[0] = u_in[0] << s;
  for (int j = nu - nv; j >= 0; j--) {
    DWord num = ((DWord)u[j + nv] << WBITS) | u[j + nv - 1];
    DWord qhat = num / v[nv - 1];
    DWord rhat = num % v[nv - 1];
    while (qhat >= ((DWord)1 << WBITS) ||
           qhat * v[nv - 2] > ((rhat << WBITS) | u[j + nv - 2])) {
      qhat--;
      rhat += v[nv - 1];
      if (rhat >= ((DWord)1 << WBITS)) break;
    }
    /* multiply and subtract */
    SDWord borrow = 0;
    DWord carry = 0;
    for (int i = 0; i < nv; i++) {
      DWord p = qhat * v[i] + carry;
      carry = p >> WBITS;
      SDWord t = (SDWord)u[i + j] - (SDWord)(Word)p + borrow;
      u[i + j] = (Word)t;
      borrow = t >> WBITS;
    }
    SDWord t = (SDWord)u[j + nv] - (SDWord)carry + borrow;
    u[j + nv] = (Word)t;
    if (t < 0) { /* add back */
      DWord c = 0;
      for (int i = 0; i < nv; i++) {
        DWord sum = (DWord)u[i + j] + v[i] + c;
        u[i + j] = (Word)sum;
        c = sum >> WBITS;
      }
      u[j + nv] += (Word)c;
    }
  }
  for (int i = 0; i < nv; i++) r[i] = s ? (u[i] >> s) | (u[i + 1] << (WBITS - s)) : u[i];
  free(u);
  free(v);
}

/* z = x*y (schoolbook), z has nx+ny words */
static void nat_mul(Word* z, const Word* x, int nx, const Word* y, int ny) {
  memset(z, 0, sizeof(Word) * (nx + ny));
  for (int i = 0; i < ny; i++) z[nx + i] = addMulVVW(z + i, x, y[i], nx);
}

/*
 * nat.montgomery: z = x*y*2^(-n*W) mod m ("almost Montgomery multiplication":
 * 0 <= z < 2^(n*W), not necessarily < m). Follows go:src/math/big/nat.go
 * (*nat).montgomery line for line, with k = -1/m mod 2^W.
 */
static void nat_montgomery(Word* z /* n */, const Word* x, const Word* y, const Word* m, Word k, int n, Word* scratch /* 2n */) {
  Word* t = scratch;
  memset(t, 0, sizeof(Word) * 2 * n);
  Word c = 0;
  for (int i = 0; i < n; i++) {
    Word d = y[i];
    Word c2 = addMulVVW(t + i, x, d, n);
    Word tt = t[i] * k;
    Word c3 = addMulVVW(t + i, m, tt, n);
    Word cx = c + c2;
    Word cy = cx + c3;
    t[n + i] = cy;
    c = (cx < c2 || cy < c3) ? 1 : 0;
  }
  if (c != 0) {
    subVV(z, t + n, m, n);
  } else {
    memcpy(z, t + n, sizeof(Word) * n);
  }
}

/* nat.expNNMontgomery (go:src/math/big/nat.go), 4-bit fixed window. */
static void nat_expNNMontgomery(Word* zout /* nm */, const Word* x_in, int nx, const Word* y, int ny, const Word* m, int nm) {
  int numWords = nm;
  Word* x = (Word*)calloc(numWords, sizeof(Word));
  nx = nat_norm(x_in, nx);
  if (nx > numWords) {
    nat_rem(x, x_in, nx, m, nm);
  } else {
    memcpy(x, x_in, sizeof(Word) * nx);
  }
  /* k0 = -m**-1 mod 2**_W (Dumas) */
  Word k0 = 2 - m[0];
  Word t = m[0] - 1;
  for (int i = 1; i < WBITS; i <<= 1) {
    t *= t;
    k0 *= (t + 1);
  }
  k0 = (Word)(-k0);
  /* RR = 2**(2*_W*len(m)) mod m */
  Word* zz2 = (Word*)calloc(2 * numWords + 1, sizeof(Word));
  zz2[2 * numWords] = 1;
  Word* RR = (Word*)calloc(numWords, sizeof(Word));
  nat_rem(RR, zz2, 2 * numWords + 1, m, nm);
  free(zz2);
  Word* one = (Word*)calloc(numWords, sizeof(Word));
  one[0] = 1;
  enum { n = 4 };
  Word* powers = (Word*)calloc((size_t)(1 << n) * numWords, sizeof(Word));
  Word* scratch = (Word*)calloc(2 * numWords, sizeof(Word));
#define PW(i) (powers + (size_t)(i) * numWords)
  nat_montgomery(PW(0), one, RR, m, k0, numWords, scratch);
  nat_montgomery(PW(1), x, RR, m, k0, numWords, scratch);
  for (int i = 2; i < (1 << n); i++) nat_montgomery(PW(i), PW(i - 1), PW(1), m, k0, numWords, scratch);
  Word* z = (Word*)calloc(numWords, sizeof(Word));
  Word* zz = (Word*)calloc(numWords, sizeof(Word));
  memcpy(z, PW(0), sizeof(Word) * numWords);
  for (int i = ny - 1; i >= 0; i--) {
    Word yi = y[i];
    for (int j = 0; j < WBITS; j += n) {
      if (i != ny - 1 || j != 0) {
        nat_montgomery(zz, z, z, m, k0, numWords, scratch);
        nat_montgomery(z, zz, zz, m, k0, numWords, scratch);
        nat_montgomery(zz, z, z, m, k0, numWords, scratch);
        nat_montgomery(z, zz, zz, m, k0, numWords, scratch);
      }
      nat_montgomery(zz, z, PW(yi >> (WBITS - n)), m, k0, numWords, scratch);
      Word* tmp = z; z = zz; zz = tmp;
      yi <<= n;
    }
  }
  nat_montgomery(zz, z, one, m, k0, numWords, scratch);
  if (nat_cmp(zz, numWords, m, numWords) >= 0) {
    subVV(zz, zz, m, numWords);
    if (nat_cmp(zz, numWords, m, numWords) >= 0) {
      Word* r = (Word*)calloc(numWords, sizeof(Word));
      nat_rem(r, zz, numWords, m, numWords);
      memcpy(zz, r, sizeof(Word) * numWords);
      free(r);
    }
  }
  memcpy(zout, zz, sizeof(Word) * numWords);
#undef PW
  free(x); free(RR); free(one); free(powers); free(scratch); free(z); free(zz);
}

/*
 * nat.expNN (go:src/math/big/nat.go): special cases, then Montgomery for odd m
 * with a multi-word (amd64: > 64-bit) exponent, else square-and-multiply with
 * a division after every step. m is assumed > 0 here (m == 0 / nil is the
 * unreduced power, unused on the hot path and rejected by go_int_exp).
 * Even m with a large exponent: Go uses expNNWindowed / expNNMontgomeryEven;
 * both return the same integer as the plain ladder below.
 * z must have room for nm words; returns the normalized length.
 */
static int nat_expNN(Word* z, const Word* x, int nx, const Word* y, int ny, const Word* m, int nm) {
  nx = nat_norm(x, nx);
  ny = nat_norm(y, ny);
  nm = nat_norm(m, nm);
  memset(z, 0, sizeof(Word) * nm);
  if (nm == 1 && m[0] == 1) return 0;                 /* x**y mod 1 == 0 */
  if (ny == 0) { z[0] = 1; return 1; }                /* x**0 == 1 */
  if (nx == 0) return 0;                              /* 0**y == 0 */
  if (nx == 1 && x[0] == 1) { z[0] = 1; return 1; }   /* 1**y == 1 */
  if (ny == 1 && y[0] == 1) {                         /* x**1 == x mod m */
    nat_rem(z, x, nx, m, nm);
    return nat_norm(z, nm);
  }
  int multiword = ny > 64 / WBITS; /* amd64 Words are 64-bit: len(y) > 1 <=> y >= 2^64 */
  if (multiword && (m[0] & 1)) {
    nat_expNNMontgomery(z, x, nx, y, ny, m, nm);
    return nat_norm(z, nm);
  }
  /* square-and-multiply, reducing mod m after each step */
  Word* zc = (Word*)calloc(nm, sizeof(Word));
  Word* xr = (Word*)calloc(nm, sizeof(Word));
  Word* prod = (Word*)calloc(2 * nm, sizeof(Word));
  nat_rem(xr, x, nx, m, nm);
  memcpy(zc, xr, sizeof(Word) * nm);
  int top = ny - 1;
  int nb = WBITS - CLZ(y[top]);
  for (int i = top; i >= 0; i--) {
    int start = (i == top) ? nb - 2 : WBITS - 1;
    for (int b = start; b >= 0; b--) {
      nat_mul(prod, zc, nm, zc, nm);
      nat_rem(zc, prod, 2 * nm, m, nm);
      if ((y[i] >> b) & 1) {
        nat_mul(prod, zc, nm, xr, nm);
        nat_rem(zc, prod, 2 * nm, m, nm);
      }
    }
  }
  memcpy(z, zc, sizeof(Word) * nm);
  free(zc); free(xr); free(prod);
  return nat_norm(z, nm);
}

/* ---------- exported entry points (test infrastructure) ---------- */

/* Unsigned x^y mod m with Go expNN semantics. out has nm words. Returns 0, or -1 if m == 0. */
EXPORT int gomodexp_expnn(Word* out, const Word* x, int nx, const Word* y, int ny, const Word* m, int nm) {
  if (nat_norm(m, nm) == 0) return -1;
  nat_expNN(out, x, nx, y, ny, m, nm);
  return 0;
}

/* Force the Montgomery path (odd m), used by the CPU baseline: same 4-bit-window
 * AMM algorithm Go runs for multi-word exponents. */
EXPORT int gomodexp_montgomery(Word* out, const Word* x, int nx, const Word* y, int ny, const Word* m, int nm) {
  if (nm <= 0 || (m[0] & 1) == 0) return -1;
  nat_expNNMontgomery(out, x, nx, y, ny, m, nm);
  return 0;
}

/* Batched Montgomery path with a shared exponent; operands are count x nm words. */
EXPORT int gomodexp_montgomery_batch(Word* out, const Word* x, int count, const Word* y, int ny, const Word* m, int nm) {
  for (int i = 0; i < count; i++) {
    int rc = gomodexp_montgomery(out + (size_t)i * nm, x + (size_t)i * nm, nm, y, ny, m, nm);
    if (rc) return rc;
  }
  return 0;
}

int gomodexp_word_bits(void) { return WBITS; }

#ifdef GOMODEXP_W64
/* 64-bit-Word build: the same entry points over little-endian 32-bit words
 * (packed into 64-bit Words on entry, unpacked on exit; n32 = 32-bit words). */
static Word* pack64(const uint32_t* x, int n32, int* n64) {
  *n64 = (n32 + 1) / 2;
  Word* w = (Word*)calloc((size_t)(*n64 > 0 ? *n64 : 1), sizeof(Word));
  for (int i = 0; i < n32; i++) w[i / 2] |= (Word)x[i] << (32 * (i % 2));
  return w;
}

static void unpack64(uint32_t* out, int n32, const Word* w) {
  for (int i = 0; i < n32; i++) out[i] = (uint32_t)(w[i / 2] >> (32 * (i % 2)));
}

int gomodexp64_montgomery(uint32_t* out, const uint32_t* x, int nx, const uint32_t* y, int ny, const uint32_t* m,
                          int nm) {
  int ax, ay, am;
  Word *X = pack64(x, nx, &ax), *Y = pack64(y, ny, &ay), *M = pack64(m, nm, &am);
  Word* Z = (Word*)calloc((size_t)am, sizeof(Word));
  int rc = gomodexp_montgomery(Z, X, ax, Y, ay, M, am);
  if (rc == 0) unpack64(out, nm, Z);
  free(X); free(Y); free(M); free(Z);
  return rc;
}

int gomodexp64_expnn(uint32_t* out, const uint32_t* x, int nx, const uint32_t* y, int ny, const uint32_t* m, int nm) {
  int ax, ay, am;
  Word *X = pack64(x, nx, &ax), *Y = pack64(y, ny, &ay), *M = pack64(m, nm, &am);
  Word* Z = (Word*)calloc((size_t)am, sizeof(Word));
  int rc = gomodexp_expnn(Z, X, ax, Y, ay, M, am);
  if (rc == 0) unpack64(out, nm, Z);
  free(X); free(Y); free(M); free(Z);
  return rc;
}
#endif
