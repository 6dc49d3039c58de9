// Shared device/host helpers for the CSE (classical speech enhancement) engine.
// gfx950 / CDNA4 only: wave64, no CUDA shims.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

#include "../../include/cse.h"

// ----------------------------------------------------------------------------
// error reporting (thread-local message behind cse_last_error())
// ----------------------------------------------------------------------------
namespace cse {

void set_error(const char* fmt, ...);

#define CSE_CHECK_ARG(cond, ...)                 \
    do {                                         \
        if (!(cond)) {                           \
            ::cse::set_error(__VA_ARGS__);       \
            return CSE_EINVAL;                   \
        }                                        \
    } while (0)

#define CSE_CHECK_LAUNCH(what)                                               \
    do {                                                                     \
        hipError_t e_ = hipGetLastError();                                   \
        if (e_ != hipSuccess) {                                              \
            ::cse::set_error("%s: %s", what, hipGetErrorString(e_));         \
            return CSE_ELAUNCH;                                              \
        }                                                                    \
    } while (0)

static inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// frames of a centred STFT of an even n_fft (librosa 0.11): 1 + len // hop
static inline int n_frames_for(int64_t len, int hop) { return 1 + (int)(len / hop); }

// ----------------------------------------------------------------------------
// complex float helpers
// ----------------------------------------------------------------------------
struct __attribute__((aligned(8))) cf {
    float x, y;
};

// e^{2πi m/32}, m = 0..31 (all the compile-time rotors the kernels need)
struct Rot32 {
    static constexpr float c[32] = {
        1.0f, 0.98078528040323043f, 0.92387953251128674f, 0.83146961230254524f,
        0.70710678118654752f, 0.55557023301960218f, 0.38268343236508978f, 0.19509032201612826f,
        0.0f, -0.19509032201612826f, -0.38268343236508978f, -0.55557023301960218f,
        -0.70710678118654752f, -0.83146961230254524f, -0.92387953251128674f, -0.98078528040323043f,
        -1.0f, -0.98078528040323043f, -0.92387953251128674f, -0.83146961230254524f,
        -0.70710678118654752f, -0.55557023301960218f, -0.38268343236508978f, -0.19509032201612826f,
        0.0f, 0.19509032201612826f, 0.38268343236508978f, 0.55557023301960218f,
        0.70710678118654752f, 0.83146961230254524f, 0.92387953251128674f, 0.98078528040323043f};
    static constexpr float s[32] = {
        0.0f, 0.19509032201612826f, 0.38268343236508978f, 0.55557023301960218f,
        0.70710678118654752f, 0.83146961230254524f, 0.92387953251128674f, 0.98078528040323043f,
        1.0f, 0.98078528040323043f, 0.92387953251128674f, 0.83146961230254524f,
        0.70710678118654752f, 0.55557023301960218f, 0.38268343236508978f, 0.19509032201612826f,
        0.0f, -0.19509032201612826f, -0.38268343236508978f, -0.55557023301960218f,
        -0.70710678118654752f, -0.83146961230254524f, -0.92387953251128674f, -0.98078528040323043f,
        -1.0f, -0.98078528040323043f, -0.92387953251128674f, -0.83146961230254524f,
        -0.70710678118654752f, -0.55557023301960218f, -0.38268343236508978f, -0.19509032201612826f};
};

__device__ __forceinline__ cf cmk(float x, float y) { return cf{x, y}; }
__device__ __forceinline__ cf cadd(cf a, cf b) { return cf{a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cf csub(cf a, cf b) { return cf{a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ cf cmul(cf a, cf b) {
    return cf{fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x)};
}
__device__ __forceinline__ cf cconj(cf a) { return cf{a.x, -a.y}; }
// multiply by +i
__device__ __forceinline__ cf cmuli(cf a) { return cf{-a.y, a.x}; }
__device__ __forceinline__ cf cscale(cf a, float s) { return cf{a.x * s, a.y * s}; }

// ----------------------------------------------------------------------------
// In-register inverse DFT of length 16 (sign +i): x[n] = sum_k X[k] e^{+2πi nk/16}
// radix-4 x radix-4: k = 4k1 + k2, n = n1 + 4n2.
// ----------------------------------------------------------------------------
__device__ __forceinline__ void idft4(cf& a0, cf& a1, cf& a2, cf& a3) {
    cf s02 = cadd(a0, a2), d02 = csub(a0, a2);
    cf s13 = cadd(a1, a3), d13 = cmuli(csub(a1, a3));
    a0 = cadd(s02, s13);
    a2 = csub(s02, s13);
    a1 = cadd(d02, d13);
    a3 = csub(d02, d13);
}

// W16^m = e^{+2πi m/16} for m in [0, 9] (n1*k2 <= 9)
__device__ __forceinline__ cf w16(int m) {
    constexpr float c1 = 0.92387953251128674f, s1 = 0.38268343236508978f;
    constexpr float r2 = 0.70710678118654752f;
    switch (m) {
        case 0: return cf{1.f, 0.f};
        case 1: return cf{c1, s1};
        case 2: return cf{r2, r2};
        case 3: return cf{s1, c1};
        case 4: return cf{0.f, 1.f};
        case 5: return cf{-s1, c1};
        case 6: return cf{-r2, r2};
        case 7: return cf{-c1, s1};
        case 8: return cf{-1.f, 0.f};
        default: return cf{-c1, -s1};  // 9
    }
}

// Second radix-4 stage of idft16 for row n1 in 1..3, the twiddles W16^{n1 k2}
// folded into FMAs.  With w = W16^{n1}, rho = w^2 and a_k2 = w^k2 b_k2:
//   s02 = b0 + rho b2, d02 = b0 - rho b2, a1 +/- a3 = w (b1 +/- rho b3) = w p / w m,
//   y0 = s02 + w p, y2 = s02 - w p, y1 = d02 + i w m, y3 = d02 - i w m.
// rho b is r2 (b.x - b.y, b.x + b.y) (n1 = 1), i b (2), r2 (-b.x - b.y, b.x - b.y) (3);
// w = c (1 + i tau) (Linzer-Feig): w p = c g with g = (p.x - tau p.y, p.y + tau p.x),
// and each +/- c g is one FMA per component.  20-24 operations per row
// instead of 24-28 (3 complex products and 16 additions).
template <int N1>
__device__ __forceinline__ void idft4_tw(cf& a0, cf& a1, cf& a2, cf& a3) {
    constexpr float r2 = 0.70710678118654752f;
    constexpr float c1 = 0.92387953251128674f, s1 = 0.38268343236508978f;
    constexpr float C = N1 == 1 ? c1 : (N1 == 2 ? r2 : s1);      // w = C (1 + i TAU)
    constexpr float TAU = N1 == 1 ? s1 / c1 : (N1 == 2 ? 1.0f : c1 / s1);
    const cf b0 = a0, b1 = a1, b2 = a2, b3 = a3;
    cf s02, d02, p, m;
    if (N1 == 2) {  // rho = i
        s02 = cmk(b0.x - b2.y, b0.y + b2.x);
        d02 = cmk(b0.x + b2.y, b0.y - b2.x);
        p = cmk(b1.x - b3.y, b1.y + b3.x);
        m = cmk(b1.x + b3.y, b1.y - b3.x);
    } else {
        const cf q2 = N1 == 1 ? cmk(b2.x - b2.y, b2.x + b2.y) : cmk(-b2.x - b2.y, b2.x - b2.y);
        const cf q3 = N1 == 1 ? cmk(b3.x - b3.y, b3.x + b3.y) : cmk(-b3.x - b3.y, b3.x - b3.y);
        s02 = cmk(fmaf(r2, q2.x, b0.x), fmaf(r2, q2.y, b0.y));
        d02 = cmk(fmaf(-r2, q2.x, b0.x), fmaf(-r2, q2.y, b0.y));
        p = cmk(fmaf(r2, q3.x, b1.x), fmaf(r2, q3.y, b1.y));
        m = cmk(fmaf(-r2, q3.x, b1.x), fmaf(-r2, q3.y, b1.y));
    }
    const cf g = N1 == 2 ? cmk(p.x - p.y, p.y + p.x) : cmk(fmaf(-TAU, p.y, p.x), fmaf(TAU, p.x, p.y));
    const cf h = N1 == 2 ? cmk(m.x - m.y, m.y + m.x) : cmk(fmaf(-TAU, m.y, m.x), fmaf(TAU, m.x, m.y));
    a0 = cmk(fmaf(C, g.x, s02.x), fmaf(C, g.y, s02.y));
    a2 = cmk(fmaf(-C, g.x, s02.x), fmaf(-C, g.y, s02.y));
    a1 = cmk(fmaf(-C, h.y, d02.x), fmaf(C, h.x, d02.y));   // d02 + i C h
    a3 = cmk(fmaf(C, h.y, d02.x), fmaf(-C, h.x, d02.y));   // d02 - i C h
}

__device__ __forceinline__ void idft16(cf (&v)[16]) {
    // step 1: for each k2, DFT4 over k1 of v[4k1+k2] -> index n1 (stored in place)
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) idft4(v[k2], v[4 + k2], v[8 + k2], v[12 + k2]);
    // now v[4*n1 + k2] holds A[n1][k2]; step 2: for each n1, DFT4 over k2 of
    // W16^{n1 k2} A[n1][k2] -> index n2; result x[n1 + 4n2]
    idft4(v[0], v[1], v[2], v[3]);
    idft4_tw<1>(v[4], v[5], v[6], v[7]);
    idft4_tw<2>(v[8], v[9], v[10], v[11]);
    idft4_tw<3>(v[12], v[13], v[14], v[15]);
    // v[4*n1 + n2] = x[n1 + 4 n2]: transpose 4x4 to natural order
    cf t[16];
#pragma unroll
    for (int n1 = 0; n1 < 4; ++n1)
#pragma unroll
        for (int n2 = 0; n2 < 4; ++n2) t[n1 + 4 * n2] = v[4 * n1 + n2];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = t[i];
}

// ----------------------------------------------------------------------------
// Packed f32 pairs.  gfx950 executes v_pk_fma/mul/add_f32 (two f32 lanes per
// instruction) at the SIMD's scalar f32 rate, but a wave issues one VALU
// instruction per 4 cycles at most: a packed instruction retires two f32
// operations in that slot, so a kernel whose few resident waves cannot keep
// the SIMD busy issues half the instructions for its pairable work.  Complex
// numbers are natural pairs (re, im); the gain kernel also pairs the two
// mirror bins (k, M - k) a lane owns.  The compiler folds lane swaps and
// broadcasts (op_sel) and whole-pair negation into the instruction; a
// negation of one lane it does not fold, so those forms are FMAs against a
// constant pair (held in SGPRs) or, for a product with a run-time rotor,
// inline assembly.
// ----------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 pdup(float s) { return f2{s, s}; }

// Forms with a negation of one lane, written out: the compiler would take a
// constant pair such as (-1, 1) from two SGPRs for each (and the kernel ran out
// of SGPRs); VOP3P's op_sel / neg_lo / neg_hi do it in the instruction.
#define CSE_PK2(name, mods)                                                \
    __device__ __forceinline__ f2 name(f2 a, f2 b) {                      \
        f2 r;                                                              \
        asm("v_pk_add_f32 %0, %1, %2 " mods : "=v"(r) : "v"(a), "v"(b)); \
        return r;                                                          \
    }
// a + i b = (a.x - b.y, a.y + b.x);  a - i b = (a.x + b.y, a.y - b.x)
CSE_PK2(p_addi, "op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]")
CSE_PK2(p_subi, "op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]")
// conj(a) + i conj(b) = (a.x + b.y, -a.y + b.x)
CSE_PK2(p_conj_addi, "op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[1,0]")
#undef CSE_PK2
// (b.x - b.y, b.x + b.y) and (-b.x - b.y, b.x - b.y): r2-scaled rho b of idft4_tw
__device__ __forceinline__ f2 p_rot1(f2 b) {
    f2 r;
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[0,1] neg_lo:[0,1]" : "=v"(r) : "v"(b));
    return r;
}
__device__ __forceinline__ f2 p_rot3(f2 b) {
    f2 r;
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[0,1] neg_lo:[1,1] neg_hi:[0,1]" : "=v"(r) : "v"(b));
    return r;
}
// c + i k b = (c.x - k b.y, c.y + k b.x) and c - i k b, k a broadcast pair of
// compile-time constants (an SGPR pair: "s" requires a wave-uniform value)
__device__ __forceinline__ f2 p_fma_i(f2 b, f2 k, f2 c) {
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[1,0,0]"
        : "=v"(r) : "v"(b), "s"(k), "v"(c));
    return r;
}
__device__ __forceinline__ f2 p_fma_mi(f2 b, f2 k, f2 c) {
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_hi:[1,0,0]"
        : "=v"(r) : "v"(b), "s"(k), "v"(c));
    return r;
}
// c + (b.x s, -b.y s) and c + (-b.x s, b.y s), s = the hi lane of g:
// X_k +/- conj(X_{M-k}) with X_{M-k} = b g.y
__device__ __forceinline__ f2 p_fma_conj_hi(f2 b, f2 g, f2 c) {
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1] neg_hi:[0,1,0]"
        : "=v"(r) : "v"(b), "v"(g), "v"(c));
    return r;
}
__device__ __forceinline__ f2 p_fms_conj_hi(f2 b, f2 g, f2 c) {
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1] neg_lo:[0,1,0]"
        : "=v"(r) : "v"(b), "v"(g), "v"(c));
    return r;
}
// complex a * w, w known at compile time: (a.x w.x - a.y w.y, a.x w.y + a.y w.x)
__device__ __forceinline__ f2 p_cmulc(f2 a, float c, float s) {
    return pfma(a.yy, f2{-s, c}, a.xx * f2{c, s});
}
// complex a * w for a run-time w: v_pk_mul_f32 + v_pk_fma_f32 whose lo lane
// reads -w.y (neg_lo)
__device__ __forceinline__ f2 p_cmul(f2 a, f2 w) {
    const f2 t = a.xx * w;  // (a.x w.x, a.x w.y)
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=v"(r)
        : "v"(a), "v"(w), "v"(t));
    return r;
}

// idft4 / idft4_tw / idft16 on packed complex values: the same operations
// as the scalar forms above, one packed instruction per complex addition or
// per FMA pair (74 instructions per DFT16 instead of 148)
__device__ __forceinline__ void idft4_pk(f2& a0, f2& a1, f2& a2, f2& a3) {
    const f2 s02 = a0 + a2, d02 = a0 - a2;
    const f2 s13 = a1 + a3, e13 = a1 - a3;
    a0 = s02 + s13;
    a2 = s02 - s13;
    a1 = p_addi(d02, e13);
    a3 = p_subi(d02, e13);
}

template <int N1>
__device__ __forceinline__ void idft4_tw_pk(f2& a0, f2& a1, f2& a2, f2& a3) {
    constexpr float r2 = 0.70710678118654752f;
    constexpr float c1 = 0.92387953251128674f, s1 = 0.38268343236508978f;
    constexpr float C = N1 == 1 ? c1 : (N1 == 2 ? r2 : s1);
    constexpr float TAU = N1 == 1 ? s1 / c1 : (N1 == 2 ? 1.0f : c1 / s1);
    const f2 b0 = a0, b1 = a1, b2 = a2, b3 = a3;
    f2 s02, d02, p, m;
    if (N1 == 2) {  // rho = i
        s02 = p_addi(b0, b2);
        d02 = p_subi(b0, b2);
        p = p_addi(b1, b3);
        m = p_subi(b1, b3);
    } else {
        // q = rho b / r2: (b.x - b.y, b.x + b.y) (N1 = 1), (-b.x - b.y, b.x - b.y) (3)
        const f2 q2 = N1 == 1 ? p_rot1(b2) : p_rot3(b2);
        const f2 q3 = N1 == 1 ? p_rot1(b3) : p_rot3(b3);
        s02 = pfma(pdup(r2), q2, b0);
        d02 = pfma(-pdup(r2), q2, b0);
        p = pfma(pdup(r2), q3, b1);
        m = pfma(-pdup(r2), q3, b1);
    }
    // g = p (1 + i TAU), h = m (1 + i TAU)
    const f2 g = N1 == 2 ? p_addi(p, p) : p_fma_i(p, pdup(TAU), p);
    const f2 h = N1 == 2 ? p_addi(m, m) : p_fma_i(m, pdup(TAU), m);
    a0 = pfma(pdup(C), g, s02);
    a2 = pfma(-pdup(C), g, s02);
    a1 = p_fma_i(h, pdup(C), d02);   // d02 + i C h
    a3 = p_fma_mi(h, pdup(C), d02);  // d02 - i C h
}

__device__ __forceinline__ void idft16_pk(f2 (&v)[16]) {
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) idft4_pk(v[k2], v[4 + k2], v[8 + k2], v[12 + k2]);
    idft4_pk(v[0], v[1], v[2], v[3]);
    idft4_tw_pk<1>(v[4], v[5], v[6], v[7]);
    idft4_tw_pk<2>(v[8], v[9], v[10], v[11]);
    idft4_tw_pk<3>(v[12], v[13], v[14], v[15]);
    f2 t[16];
#pragma unroll
    for (int n1 = 0; n1 < 4; ++n1)
#pragma unroll
        for (int n2 = 0; n2 < 4; ++n2) t[n1 + 4 * n2] = v[4 * n1 + n2];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = t[i];
}

// In-register inverse DFT of length 8 on packed complex values (sign +i):
// radix-2 over the even / odd inputs, x[s] = E[s] + W8^s O[s], x[s + 4] =
// E[s] - W8^s O[s] with W8 = e^{2πi/8}: W8^1 O = r2 (o.x - o.y, o.x + o.y),
// W8^2 O = i O, W8^3 O = r2 (-o.x - o.y, o.x - o.y); 26 instructions.
__device__ __forceinline__ void idft8_pk(f2 (&v)[8]) {
    constexpr float r2 = 0.70710678118654752f;
    idft4_pk(v[0], v[2], v[4], v[6]);  // E[0..3] in v[0], v[2], v[4], v[6]
    idft4_pk(v[1], v[3], v[5], v[7]);  // O[0..3] in v[1], v[3], v[5], v[7]
    const f2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
    const f2 o0 = v[1], o1 = p_rot1(v[3]), o2 = v[5], o3 = p_rot3(v[7]);
    v[0] = e0 + o0;
    v[4] = e0 - o0;
    v[1] = pfma(pdup(r2), o1, e1);
    v[5] = pfma(-pdup(r2), o1, e1);
    v[2] = p_addi(e2, o2);
    v[6] = p_subi(e2, o2);
    v[3] = pfma(pdup(r2), o3, e3);
    v[7] = pfma(-pdup(r2), o3, e3);
}

}  // namespace cse
