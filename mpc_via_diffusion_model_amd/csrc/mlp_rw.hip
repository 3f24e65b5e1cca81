// Persistent CFG-DDPM / DDIM sampler for the MLP noise-net, fp32-accurate split-bf16
// GEMMs, with the three 128x128 layers' weights RESIDENT in registers for the whole launch.
//
// Why (profiles/r3_mlp_vmem_ab.txt): the streaming kernel (mlp_x3.hip) re-reads every
// layer's three-plane weights from L2 each denoise step, 888 KB per CU per step, and that per-CU
// vector-memory stream - not L2 bandwidth, not MFMA - sets its step time. A CU's register file is
// 512 KiB (4 SIMDs x 512 registers x 64 lanes x 4 B): with one wave per SIMD (4 waves, 512 registers
// each) the 288 KiB of Linear 5/6/7 (K = N = 128; wave w owns n-tiles w and w + 4: 24 fragments of
// 16 B per lane per layer) stay in registers across all denoise steps - 63 fragments in AGPRs, read
// directly as the MFMA A operand, 9 in VGPRs. Every other layer streams once per CU per step (each
// fragment loaded by the one wave that uses it, except the N = 32 layers at 32 rows, split by column
// tile: 324 KB per CU per step instead of 888).
//
// Same pack, LDS layout, layer order, MFMA order (six partial products of each 32-k chunk, smallest
// first, k-chunks in order, accumulators initialised from the bias / cond tables), Mish, split and
// denoise update as mlp_x3_kernel, so its results are bit-identical to the streaming kernel's
// (tests/test_gpu_mlp.py checks it).
#include <hip/hip_runtime.h>

#include "mlp_x3.h"

namespace {
using namespace mlpx3;
static_assert(WPL == 3, "mlp_rw streams the three-plane pack");

constexpr int RW_W = 4;           // waves per workgroup (one per SIMD, 512 registers each)
constexpr int RW_T = 64 * RW_W;   // threads
constexpr int RES_L0 = 5;         // resident layers 5, 6, 7
constexpr int RES_NL = 3;
constexpr int RES_G = RES_NL * 2 * 4;  // groups (layer, n-tile j, k-chunk) of 3 plane fragments per wave: 24
constexpr int RES_AG = 21;             // groups 0..20 resident in AGPRs (63 fragments, 252 registers); the
                                       // last three (layer 7, n-tile w + 4, k-chunks 1-3) stream each step

// Six partial products of one 32-k chunk with the weight planes in AGPRs (the A operand of an MFMA may be
// an AGPR on gfx950; hipcc does not allocate builtin operands there, so the chain is written out). One
// statement of six dependent MFMAs: back-to-back srcC forwarding of the same opcode needs no wait states
// (hipcc emits none between the builtin form of this chain). The leading s_nop covers a VALU write of
// acc right before the statement (the 2-wait-state VALU-write -> MFMA-read rule, which the compiler's
// hazard pass does not apply to inline asm); the MFMA result -> VALU read wait after the statement is
// inserted by the compiler (checked in tests/test_isa.py).
MPCD_DEV f32x4 mfma_x3_agpr(const u32x4 &w0, const u32x4 &w1, const u32x4 &w2, const u32x4 (&x)[3], f32x4 acc)
{
    asm("s_nop 1\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %3, %4, %0\n\t"   // w2 x0
        "v_mfma_f32_16x16x32_bf16 %0, %2, %5, %0\n\t"   // w1 x1
        "v_mfma_f32_16x16x32_bf16 %0, %1, %6, %0\n\t"   // w0 x2
        "v_mfma_f32_16x16x32_bf16 %0, %2, %4, %0\n\t"   // w1 x0
        "v_mfma_f32_16x16x32_bf16 %0, %1, %5, %0\n\t"   // w0 x1
        "v_mfma_f32_16x16x32_bf16 %0, %1, %4, %0\n\t"  // w0 x0
        "s_nop 7"                                        // result -> VALU read (see mfma_agpr1)
        : "+v"(acc)
        : "a"(w0), "a"(w1), "a"(w2), "v"(x[0]), "v"(x[1]), "v"(x[2]));
    return acc;
}

// Transcendental pairs for packed consumers: both issued, then 2 wait states before a packed op may read them (a
// packed read one wait state behind a v_exp / v_rcp gave wrong results on gfx950: unet_fused.hip exp2_pair,
// profiles/r3_hazard_ab.txt). The same instructions as __builtin_amdgcn_exp2f / rcpf: the same bits.
MPCD_DEV f32x2 exp2_pair(f32x2 z)
{
    float a, b;
    asm("v_exp_f32 %0, %2\n\tv_exp_f32 %1, %3\n\ts_nop 1" : "=&v"(a), "=&v"(b) : "v"(z[0]), "v"(z[1]));
    return f32x2{a, b};
}
MPCD_DEV f32x2 rcp_pair(f32x2 x)
{
    float a, b;
    asm("v_rcp_f32 %0, %2\n\tv_rcp_f32 %1, %3\n\ts_nop 1" : "=&v"(a), "=&v"(b) : "v"(x[0]), "v"(x[1]));
    return f32x2{a, b};
}
MPCD_DEV f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

// partial product m of a 32-k chunk, smallest first (mlp_x3.h mfma_x3): weight plane, activation plane
constexpr int wpl(int m) { return m == 0 ? 2 : (m == 1 || m == 3) ? 1 : 0; }
constexpr int xpl(int m) { return (m == 0 || m == 3 || m == 5) ? 0 : (m == 1 || m == 4) ? 1 : 2; }

// One partial product with the weight plane in an AGPR. The compiler's hazard pass does not see an MFMA in an
// asm statement, so its waits are written here: FIRST (the chain's first product), 2 wait states for a VALU
// write of the accumulator just before; LAST (the chain's last product), 8 wait states after it, before any
// VALU op may read the result (what hipcc inserts after the builtin v_mfma_f32_16x16x32_bf16 on gfx950).
// Inside a chain the accumulator goes MFMA to MFMA (srcC forwarding, no wait). tests/test_isa.py checks both
// rules on every MFMA of the library.
template <bool FIRST, bool LAST>
MPCD_DEV f32x4 mfma_agpr1(const u32x4 &w, const u32x4 &x, f32x4 acc)
{
    if constexpr (FIRST && LAST)
        asm("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\ts_nop 7" : "+v"(acc) : "a"(w), "v"(x));
    else if constexpr (FIRST)
        asm("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "a"(w), "v"(x));
    else if constexpr (LAST)
        asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\ts_nop 7" : "+v"(acc) : "a"(w), "v"(x));
    else
        asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "a"(w), "v"(x));
    return acc;
}

// MPCD_RW_ILV = 1: each hidden layer as a pipeline of passes (one n-tile x one column tile: a chain of 6 KC
// MFMAs), the previous pass's epilogue (4 Mish, the split, 3 LDS stores) issued one unit after each of this
// pass's first MFMAs (pinned with sched_barrier: a bf16 MFMA leaves the SIMD's vector issue free for 8 of its
// 16 cycles), the next activation fragments read two k-chunks ahead; 0 = the plain form (hidden()).
#ifndef MPCD_RW_ILV
#define MPCD_RW_ILV 1
#endif
// MPCD_RW_PF: k-chunks of operand fragments read ahead of the MFMAs in hidden_ilv (2: a ring of three)
#ifndef MPCD_RW_PF
#define MPCD_RW_PF 2
#endif
// MPCD_RW_TABLE_EARLY = 1: the next step's cond tables (TPC / TPU) are written after Linear 11 (the last layer that
// reads them) instead of at the step's start, where their LDS round trip delayed Linear 0's first operand reads
#ifndef MPCD_RW_TABLE_EARLY
#define MPCD_RW_TABLE_EARLY 1
#endif
// MPCD_RW_W8_SPLIT = 1 (default): Linear 8's streamed fragments issued half in Linear 5's MFMA slots, half in
// Linear 6's (0: all 24 in Linear 6's; profiles/r6_mlp_tuning_ab.txt)
#ifndef MPCD_RW_W8_SPLIT
#define MPCD_RW_W8_SPLIT 1
#endif
// MPCD_RW_TABLE_SIDE = 1 (default, with TABLE_EARLY): the table's two reads and its write ride in Linear 12's
// MFMA slots
#ifndef MPCD_RW_TABLE_SIDE
#define MPCD_RW_TABLE_SIDE 1
#endif
// MPCD_RW_PKTAIL = 1 (default): the exposed epilogue of a layer's last pass (nothing left to hide it under) with two
// values per packed instruction (v_pk_mul / v_pk_add / v_pk_fma_f32, the same roundings) instead of the fenced scalar
// micro-steps: loop VALU 1,631 -> 1,459 per wave-step, kernel -0.5 % (profiles/r6_mlp_tuning_ab.txt)
#ifndef MPCD_RW_PKTAIL
#define MPCD_RW_PKTAIL 1
#endif
// MPCD_RW_XREG = 1 (default): each lane keeps its x_t quads in registers across steps (the fp32 copy in LDS goes),
// and the update's x-only products (a x, c2 x, std z) are formed while the final layer's operand reads are in
// flight. Together with TABLE_SIDE: kernel 1.098 -> 1.090 ms at cfg2 (profiles/r6_mlp_tuning_ab.txt, 3 repeats)
#ifndef MPCD_RW_XREG
#define MPCD_RW_XREG 1
#endif
// MPCD_RW_EPI_STEPS = 1: the epilogue spread as 1-2 VALU ops per MFMA slot (hidden_ilv); 0: five units
#ifndef MPCD_RW_EPI_STEPS
#define MPCD_RW_EPI_STEPS 1
#endif

// timing experiments (wrong results): MPCD_RW_EXP_NOLASTEPI drops the last-pass epilogue of the multi-pass
// layers (hidden_ilv); MPCD_RW_EXP_BAR2 doubles every layer barrier (profiles/r4_mlp_defer_ab.txt)
#ifndef MPCD_RW_EXP_NOLASTEPI
#define MPCD_RW_EXP_NOLASTEPI 0
#endif
#ifndef MPCD_RW_EXP_BAR2
#define MPCD_RW_EXP_BAR2 0
#endif
// MPCD_RW_EXP_NOVM: the streamed layers' buffer descriptor has zero records (every streamed weight load returns 0
// without a memory access): the cost of the per-step weight stream, read as cycles per step in an MPCD_PROF_LAYERS
// build (zero operands also raise the clock, so wall time would overstate it)
#ifndef MPCD_RW_EXP_NOVM
#define MPCD_RW_EXP_NOVM 0
#endif
#if !defined(MPCD_VARIANT) && (MPCD_RW_EXP_NOLASTEPI || MPCD_RW_EXP_BAR2 || MPCD_RW_EXP_NOVM || defined(MPCD_PROF_FINAL_MFMA_ONLY))
#error "wrong-result timing switches build only as an experiment variant (build.py variant: -DMPCD_VARIANT)"
#endif

template <int D0, int SMODE, bool CTX, int R>
struct MlpRw {
    static constexpr int NB = (SMODE == MODE_DDIM || SMODE == MODE_EPS1) ? 1 : 2;
    static constexpr bool IS_DDPM = SMODE == MODE_DDPM_CFG || SMODE == MODE_DDPM_XN;
    static_assert(R == 32 || R == 16, "32 or 16 rows per workgroup");
    static constexpr int NCT = R / 16;  // 16-row column tiles
    using A = Arch<D0>;
    using L = Lds3<D0, NB, R>;
    static constexpr int CPW = L::CPW;
    static constexpr int QUADS = D0 / 4;

    // Row swizzle of every activation plane (as mlp_h2.hip's Lds2): in rows with bit 2 set the 16-byte units are
    // swapped in pairs (byte offset b -> b ^ 16). The B-fragment reads (ds_read_b128 of whole units, lane (col, q)
    // reading unit q ^ s of its row) stay conflict-free; the epilogue's ds_write_b64 of 16 rows at one feature
    // offset (one lane group, banks mod 32) drop from 4-way to 2-way bank conflicts - 2-way is that pattern's
    // floor (16 rows on the 8 unit positions of 128 bytes). s = bit 2 of the row = bit 2 of the lane's column in
    // every layout here (rows ct * 16 + col, or the candidate col / col & 7 of the shared layer-0 input).
    static MPCD_DEV int swz(int r) { return (r >> 2) & 1; }
    // byte offset in its row of the 4 features n..n+3 (n = 16 nt + 4 q) an epilogue lane of quarter q stores
    static MPCD_DEV int st_off(int n, int q, int row) { return n * 2 - 8 * q + 8 * (q ^ (swz(row) << 1)); }

    // R = 16 with CFG: columns 0-7 are the context rows of candidates 0-7, 8-15 their masked rows
    static MPCD_DEV int cand_of(int ct, int col) { return NB == 2 ? (R == 16 ? (col & 7) : col) : ct * 16 + col; }
    static MPCD_DEV bool masked_of(int ct, int col) { return NB == 2 && (R == 16 ? col >= 8 : ct == 1); }

    // Layer l's work per wave. N = 32 at 32 rows (SPL): wave w -> n-tile w & 1, column tile w >> 1. Otherwise
    // wave w -> n-tiles w + 4j (j < T) for every column tile; a wave with no tile (N = 32 at 16 rows) loads
    // a clamped copy and computes nothing.
    template <int l> static constexpr bool SPL = A::N[l] == 32 && NCT == 2;
    template <int l> static constexpr int TL = SPL<l> ? 1 : (A::N[l] / 16 + 3) / 4;
    template <int l> static constexpr int CL = SPL<l> ? 1 : NCT;
    template <int l> static MPCD_DEV int nt_of(int wave, int j) { return SPL<l> ? (wave & 1) : wave + 4 * j; }
    template <int l> static MPCD_DEV int ct_of(int wave, int c) { return SPL<l> ? (wave >> 1) : c; }

    // ONE buffer descriptor over the whole weight pack for every streamed layer (the layer offset goes into the
    // soffset): per-layer descriptors, kept live across the step loop, cost 4 SGPRs each and pushed ~50 SGPRs into
    // VGPR lanes (a v_readlane per use)
    static MPCD_DEV __amdgpu_buffer_rsrc_t pack_rsrc(const float *__restrict__ wp)
    {
        const uint64_t a = (uint64_t)wp;
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
        return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0,
                                                 MPCD_RW_EXP_NOVM ? 0 : (int)(woffx<D0>(NLAYER) * 4), 0x00020000);
    }

    // streamed fragments of layer l for this wave
    template <int l>
    struct WS {
        u32x4 v[TL<l>][A::K[l] / 32][3];
    };

    template <int l>
    static MPCD_DEV void load_ws(WS<l> &f, const float *__restrict__ wp, int wave, int lane16)
    {
        constexpr int K = A::K[l], N = A::N[l], KC = K / 32, NT = N / 16;
        const __amdgpu_buffer_rsrc_t rs = pack_rsrc(wp);
#pragma unroll
        for (int j = 0; j < TL<l>; ++j) {
            const int nt = min(nt_of<l>(wave, j), NT - 1);  // clamped: path-independent load count
#pragma unroll
            for (int kc = 0; kc < KC; ++kc)
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) {
                    const int soff = __builtin_amdgcn_readfirstlane(woffx<D0>(l) * 4 + ((nt * KC + kc) * 3 + pl) * 1024);
                    f.v[j][kc][pl] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane16, soff, 0));
                }
        }
    }

    // fragment f (= (j * KC + kc) * 3 + plane) of layer l for this wave: load_ws one piece at a time, issued in
    // the free MFMA slots of an earlier layer (hidden_ilv's side work)
    template <int l>
    static MPCD_DEV void load_ws1(WS<l> &w, const float *__restrict__ wp, int wave, int lane16, int f)
    {
        constexpr int K = A::K[l], N = A::N[l], KC = K / 32, NT = N / 16;
        const __amdgpu_buffer_rsrc_t rs = pack_rsrc(wp);
        const int j = f / (KC * 3), kc = (f / 3) % KC, pl = f % 3;
        const int nt = min(nt_of<l>(wave, j), NT - 1);
        const int soff = __builtin_amdgcn_readfirstlane(woffx<D0>(l) * 4 + ((nt * KC + kc) * 3 + pl) * 1024);
        w.v[j][kc][pl] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane16, soff, 0));
    }
    template <int l>
    static constexpr int NFRAG = TL<l> * (A::K[l] / 32) * 3;

    // Resident fragments: group g = ((li * 2 + j) * 4 + kc), planes 0..2 (AGPRs); Tail: groups RES_AG.. of
    // layer 7, streamed like the other layers (VGPRs)
    struct Res {
        u32x4 a[RES_AG][3];
    };
    struct Tail {
        u32x4 v[RES_G - RES_AG][3];
    };
    static MPCD_DEV void load_tail1(Tail &t, const float *__restrict__ wp, int wave, int lane16, int f)
    {
        const __amdgpu_buffer_rsrc_t rs = pack_rsrc(wp);
        const int g = RES_AG + f / 3, pl = f % 3, j = (g / 4) & 1, kc = g & 3, nt = wave + 4 * j;
        const int soff = __builtin_amdgcn_readfirstlane(woffx<D0>(RES_L0 + RES_NL - 1) * 4 + ((nt * 4 + kc) * 3 + pl) * 1024);
        t.v[g - RES_AG][pl] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane16, soff, 0));
    }
    static MPCD_DEV void load_tail(Tail &t, const float *__restrict__ wp, int wave, int lane16)
    {
        const __amdgpu_buffer_rsrc_t rs = pack_rsrc(wp);
#pragma unroll
        for (int g = RES_AG; g < RES_G; ++g) {
            const int j = (g / 4) & 1, kc = g & 3, nt = wave + 4 * j;
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) {
                const int soff = __builtin_amdgcn_readfirstlane(woffx<D0>(RES_L0 + RES_NL - 1) * 4 + ((nt * 4 + kc) * 3 + pl) * 1024);
                t.v[g - RES_AG][pl] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane16, soff, 0));
            }
        }
    }

    static MPCD_DEV void load_res(Res &r, const float *__restrict__ wp, int wave, int lane)
    {
#pragma unroll
        for (int g = 0; g < RES_AG; ++g) {
            const int li = g / 8, j = (g / 4) & 1, kc = g & 3;
            const int nt = wave + 4 * j;
            const float *base = wp + woffx<D0>(RES_L0 + li) + (size_t)((nt * 4 + kc) * 3) * 256 + lane * 4;
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) {
                r.a[g][pl] = __builtin_bit_cast(u32x4, ldg4(base + pl * 256));
            }
        }
    }

    // Hidden layer l: per n-tile pass j, k-chunks in order over this wave's column tiles; pass j's epilogue
    // (Mish, 3-way split, LDS stores of the next layer's operand planes) is issued behind pass j + 1's MFMAs.
    // MM(j, kc, x[3], acc) -> acc: the six partial products with this wave's fragments of (j, kc).
    template <int l, class MM>
    static MPCD_DEV void hidden(MM mm, char *lds, int wave, int lane)
    {
        constexpr int K = A::K[l], N = A::N[l], KC = K / 32, NT = N / 16, T = TL<l>, NC = CL<l>, EPI = epi_of(l);
        const int col = lane & 15, q = lane >> 4;
        constexpr bool in_shared = l == 0 && NB == 2;  // CFG: both branches read the candidate's x
        static_assert(T == 1 || NT % 4 == 0, "only a one-tile layer can leave a wave idle");
        if constexpr (NT < 4 && !SPL<l>)
            if (wave >= NT) return;  // N = 32 at 16 rows: waves 2, 3 have no tile
        f32x4 acc[T][NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int ct = ct_of<l>(wave, c);
            const float *init = reinterpret_cast<const float *>(
                lds + (EPI == EPI_CMISH ? (masked_of(ct, col) ? L::TPU : L::TPC) + cond_off(l / 2) * 4
                                        : L::BI + A::boff(l) * 4));
#pragma unroll
            for (int j = 0; j < T; ++j)
                acc[j][c] = *reinterpret_cast<const f32x4 *>(init + min(nt_of<l>(wave, j), NT - 1) * 16 + 4 * q);
        }
        auto ldx = [&](u32x4 (&x)[NC][3], int kc) {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int ct = ct_of<l>(wave, c);
                const int row = in_shared ? cand_of(ct, col) : ct * 16 + col;
                load_x3(x[c], lds + L::in_off(l) + row * L::in_rs(l) + kc * 64 + 16 * (q ^ swz(row)), L::in_pl(l));
            }
        };
        auto epi = [&](int j, int c) {
            const int n = nt_of<l>(wave, j) * 16 + 4 * q;
            f32x4 v = acc[j][c];
            if (EPI != EPI_NONE) {
                v.x = mish_scalar(v.x);
                v.y = mish_scalar(v.y);
                v.z = mish_scalar(v.z);
                v.w = mish_scalar(v.w);
            }
            u32x2 p0, p1, p2;
            split3(v, p0, p1, p2);
            const int ro = ct_of<l>(wave, c) * 16 + col;
            char *o = lds + L::out_off(l) + ro * L::out_rs(l) + st_off(n, q, ro);
            *reinterpret_cast<u32x2 *>(o) = p0;
            *reinterpret_cast<u32x2 *>(o + L::out_pl(l)) = p1;
            *reinterpret_cast<u32x2 *>(o + 2 * L::out_pl(l)) = p2;
        };
#pragma unroll
        for (int j = 0; j < T; ++j) {
            u32x4 xc[NC][3], xn[NC][3];
            ldx(xc, 0);
#pragma unroll
            for (int kc = 0; kc < KC; ++kc) {
                if (kc + 1 < KC) ldx(xn, kc + 1);
#pragma unroll
                for (int c = 0; c < NC; ++c) acc[j][c] = mm(j, kc, xc[c], acc[j][c]);
                if (j > 0 && kc == 0) {
                    // the previous pass's epilogue in this pass's MFMA shadow
#pragma unroll
                    for (int c = 0; c < NC; ++c) epi(j - 1, c);
                }
                if (kc + 1 < KC)
#pragma unroll
                    for (int c = 0; c < NC; ++c)
#pragma unroll
                        for (int pl = 0; pl < 3; ++pl) xc[c][pl] = xn[c][pl];
            }
            if (j == T - 1)
#pragma unroll
                for (int c = 0; c < NC; ++c) epi(j, c);
        }
    }

    // Pipelined form of hidden(). MM1(j, kc, m, x[3], acc) -> acc: partial product m (0..5, smallest first:
    // the mfma_x3 order) of k-chunk kc of n-tile j. Same products in the same order as hidden(): bit-identical.
    // free MFMA slots of layer l's pipeline (the first 5 of every pass but the first carry epilogue units)
    template <int l>
    static constexpr int FREE = TL<l> * CL<l> * (A::K[l] / 32) * 6 - 5 * (TL<l> * CL<l> - 1);

    // SIDE(k), k < NS: side work, one item per free slot in order; items beyond the free slots (and all of them
    // on a wave with no tile) run after the layer's MFMAs
    template <int l, int NS, class MM1, class SIDE>
    static MPCD_DEV void hidden_ilv(MM1 mm1, SIDE side, char *lds, int wave, int lane)
    {
        constexpr int K = A::K[l], N = A::N[l], KC = K / 32, NT = N / 16, T = TL<l>, NC = CL<l>, EPI = epi_of(l);
        constexpr int NP = T * NC, NI = NP * KC;  // passes; (pass, k-chunk) steps
        const int col = lane & 15, q = lane >> 4;
        constexpr bool in_shared = l == 0 && NB == 2;  // CFG: both branches read the candidate's x
        static_assert(T == 1 || NT % 4 == 0, "only a one-tile layer can leave a wave idle");
        if constexpr (NT < 4 && !SPL<l>)
            if (wave >= NT) {  // N = 32 at 16 rows: waves 2, 3 have no tile
#pragma unroll
                for (int k = 0; k < NS; ++k) side(k);
                return;
            }
        auto jp = [](int p) { return p / NC; };
        auto cp = [](int p) { return p % NC; };
        auto init_of = [&](int p) {
            const int ct = ct_of<l>(wave, cp(p));
            const float *init = reinterpret_cast<const float *>(
                lds + (EPI == EPI_CMISH ? (masked_of(ct, col) ? L::TPU : L::TPC) + cond_off(l / 2) * 4
                                        : L::BI + A::boff(l) * 4));
            return *reinterpret_cast<const f32x4 *>(init + min(nt_of<l>(wave, jp(p)), NT - 1) * 16 + 4 * q);
        };
        auto ldx = [&](u32x4 (&x)[3], int i) {  // step i = (pass i / KC, k-chunk i % KC)
            const int p = i / KC, kc = i % KC, ct = ct_of<l>(wave, cp(p));
            const int row = in_shared ? cand_of(ct, col) : ct * 16 + col;
            load_x3(x, lds + L::in_off(l) + row * L::in_rs(l) + kc * 64 + 16 * (q ^ swz(row)), L::in_pl(l));
        };
        // epilogue of pass p in five units: Mish of element 0..3, then the split + the three plane stores
        auto epi_unit = [&](int u, f32x4 &v, int p) {
            if (u < 4) {
                if (EPI != EPI_NONE) v[u] = mish_scalar(v[u]);
                return;
            }
            const int n = nt_of<l>(wave, jp(p)) * 16 + 4 * q;
            u32x2 p0, p1, p2;
            split3(v, p0, p1, p2);
            const int ro = ct_of<l>(wave, cp(p)) * 16 + col;
            char *o = lds + L::out_off(l) + ro * L::out_rs(l) + st_off(n, q, ro);
            *reinterpret_cast<u32x2 *>(o) = p0;
            *reinterpret_cast<u32x2 *>(o + L::out_pl(l)) = p1;
            *reinterpret_cast<u32x2 *>(o + 2 * L::out_pl(l)) = p2;
        };
        // operand fragments read PF k-chunks ahead (a ring of PF + 1)
        constexpr int PF = MPCD_RW_PF;
        u32x4 xb[PF + 1][3];
#pragma unroll
        for (int i = 0; i < PF; ++i)
            if (i < NI) ldx(xb[i], i);
        f32x4 acc = init_of(0), nxt = acc, ev = acc;
#if MPCD_RW_EPI_STEPS
        // The previous pass's epilogue as NSTEP micro-steps of one or two VALU instructions, one after each MFMA:
        // a bf16 MFMA leaves the SIMD's vector issue free for 8 of its 16 cycles, i.e. about two VALU ops. Stage
        // by stage over the four values (the dependent ops of one value 4 slots apart), the exact operations of
        // common.h mish() and split3(); every intermediate through an empty register fence (no SLP packing).
        float et[4];
        u32x2 ep0, ep1, ep2;
        float er0 = 0.f, er1 = 0.f, er2 = 0.f, er3 = 0.f;
        constexpr int NSTEP = (EPI != EPI_NONE ? 16 : 0) + 8;
        auto fence = [](float &x) { asm volatile("" : "+v"(x)); };
        auto epi_step = [&](int k, int p) {
            if (EPI != EPI_NONE && k < 16) {
                const int e = k & 3;
                switch (k >> 2) {
                case 0: et[e] = __builtin_amdgcn_exp2f(ev[e] * 1.44269504088896341f); fence(et[e]); break;
                case 1: et[e] = __builtin_fmaf(et[e], et[e] + 2.0f, 2.0f); fence(et[e]); break;
                case 2: et[e] = __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(et[e]), 1.0f); fence(et[e]); break;
                default: { float y = ev[e] * et[e]; fence(y); ev[e] = y; } break;
                }
                return;
            }
            const int s = EPI != EPI_NONE ? k - 16 : k;
            const int n = nt_of<l>(wave, jp(p)) * 16 + 4 * q;
            const int ro = ct_of<l>(wave, cp(p)) * 16 + col;
            char *o = lds + L::out_off(l) + ro * L::out_rs(l) + st_off(n, q, ro);
            switch (s) {  // split3 (mlp_x3.h), in pieces
            // each remainder through a fence: the compiler would otherwise pair the two subtractions of a step
            // into one v_pk_add_f32, which beside MFMAs costs more issue time than the two plain ones
            // (MI355X_MICROARCH.md, price of one filler beside MFMAs)
            case 0: ep0 = u32x2{pk_bf16(ev.x, ev.y), pk_bf16(ev.z, ev.w)}; break;
            case 1: er0 = ev.x - bf_lo(ep0.x); fence(er0); er1 = ev.y - bf_hi(ep0.x); fence(er1); break;
            case 2: er2 = ev.z - bf_lo(ep0.y); fence(er2); er3 = ev.w - bf_hi(ep0.y); fence(er3); *reinterpret_cast<u32x2 *>(o) = ep0; break;
            case 3: ep1 = u32x2{pk_bf16(er0, er1), pk_bf16(er2, er3)}; break;
            case 4: er0 = er0 - bf_lo(ep1.x); fence(er0); er1 = er1 - bf_hi(ep1.x); fence(er1); break;
            case 5: er2 = er2 - bf_lo(ep1.y); fence(er2); er3 = er3 - bf_hi(ep1.y); fence(er3); break;
            case 6: *reinterpret_cast<u32x2 *>(o + L::out_pl(l)) = ep1; ep2 = u32x2{pk_bf16(er0, er1), pk_bf16(er2, er3)}; break;
            default: *reinterpret_cast<u32x2 *>(o + 2 * L::out_pl(l)) = ep2; break;
            }
        };
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            if (p + 1 < NP) nxt = init_of(p + 1);
#pragma unroll
            for (int kc = 0; kc < KC; ++kc) {
                const int i = p * KC + kc;
                if (i + PF < NI) ldx(xb[(i + PF) % (PF + 1)], i + PF);
#pragma unroll
                for (int m = 0; m < 6; ++m) {
                    acc = mm1(jp(p), kc, m, xb[i % (PF + 1)], acc);
                    const int u = kc * 6 + m;
                    if (p > 0 && u < NSTEP) epi_step(u, p - 1);
                    if (i * 6 + m < NS) side(i * 6 + m);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            if (p > 0)
#pragma unroll
                for (int u = KC * 6; u < NSTEP; ++u) epi_step(u, p - 1);  // passes shorter than the epilogue
            ev = acc;
            acc = nxt;
        }
        // the last pass's epilogue, exposed (MPCD_RW_PKTAIL: packed, two values per instruction; epi_step's operations)
        auto epi_tail = [&](int p) {
            f32x2 a = {ev[0], ev[1]}, b = {ev[2], ev[3]};
            if constexpr (EPI != EPI_NONE) {
                const f32x2 l2e = {1.44269504088896341f, 1.44269504088896341f}, two = {2.0f, 2.0f};
                const f32x2 m2 = {-2.0f, -2.0f}, one = {1.0f, 1.0f};
                f32x2 ta = exp2_pair(a * l2e), tb = exp2_pair(b * l2e);
                ta = fma2(ta, ta + two, two);
                tb = fma2(tb, tb + two, two);
                ta = fma2(m2, rcp_pair(ta), one);
                tb = fma2(m2, rcp_pair(tb), one);
                a = a * ta;
                b = b * tb;
            }
            const int n = nt_of<l>(wave, jp(p)) * 16 + 4 * q;
            const int ro = ct_of<l>(wave, cp(p)) * 16 + col;
            char *o = lds + L::out_off(l) + ro * L::out_rs(l) + st_off(n, q, ro);
            const u32x2 q0 = {pk_bf16(a[0], a[1]), pk_bf16(b[0], b[1])};
            *reinterpret_cast<u32x2 *>(o) = q0;
            a = a - f32x2{bf_lo(q0.x), bf_hi(q0.x)};
            b = b - f32x2{bf_lo(q0.y), bf_hi(q0.y)};
            const u32x2 q1 = {pk_bf16(a[0], a[1]), pk_bf16(b[0], b[1])};
            *reinterpret_cast<u32x2 *>(o + L::out_pl(l)) = q1;
            a = a - f32x2{bf_lo(q1.x), bf_hi(q1.x)};
            b = b - f32x2{bf_lo(q1.y), bf_hi(q1.y)};
            *reinterpret_cast<u32x2 *>(o + 2 * L::out_pl(l)) = u32x2{pk_bf16(a[0], a[1]), pk_bf16(b[0], b[1])};
        };
        // MPCD_RW_EXP_NOLASTEPI (timing experiment only, wrong results): drop the exposed last-pass epilogue of
        // the multi-pass layers - the bound on what deferring it into the next layer could gain
        if (!(MPCD_RW_EXP_NOLASTEPI && NP >= 2)) {
            if constexpr (MPCD_RW_PKTAIL) {
                epi_tail(NP - 1);
            } else {
#pragma unroll
                for (int u = 0; u < NSTEP; ++u) epi_step(u, NP - 1);
            }
        }
#pragma unroll
        for (int k = NI * 6; k < NS; ++k) side(k);
#else
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            if (p + 1 < NP) nxt = init_of(p + 1);
#pragma unroll
            for (int kc = 0; kc < KC; ++kc) {
                const int i = p * KC + kc;
                if (i + PF < NI) ldx(xb[(i + PF) % (PF + 1)], i + PF);
#pragma unroll
                for (int m = 0; m < 6; ++m) {
                    acc = mm1(jp(p), kc, m, xb[i % (PF + 1)], acc);
                    const int u = kc * 6 + m;
                    if (p > 0 && u < 5) epi_unit(u, ev, p - 1);
                    else if (i * 6 + m - 5 * p < NS) side(i * 6 + m - 5 * p);  // the k-th free slot
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            ev = acc;
            acc = nxt;
        }
#pragma unroll
        for (int u = 0; u < 5; ++u) epi_unit(u, ev, NP - 1);
#pragma unroll
        for (int k = FREE<l>; k < NS; ++k) side(k);
#endif
    }

    template <int l, int NS = 0, class SIDE>
    static MPCD_DEV void layer(const WS<l> &w, SIDE side, char *lds, int wave, int lane)
    {
#if MPCD_RW_ILV
        hidden_ilv<l, NS>(
            [&](int j, int kc, int m, const u32x4 (&x)[3], f32x4 acc) { return mfma_bf(w.v[j][kc][wpl(m)], x[xpl(m)], acc); },
            side, lds, wave, lane);
#else
        hidden<l>([&](int j, int kc, const u32x4 (&x)[3], f32x4 acc) { return mfma_x3(w.v[j][kc], x, acc); }, lds, wave,
                  lane);
#pragma unroll
        for (int k = 0; k < NS; ++k) side(k);
#endif
    }

    template <int li, int NS = 0, class SIDE>
    static MPCD_DEV void layer_res(const Res &r, const Tail &t, SIDE side, char *lds, int wave, int lane)
    {
#if MPCD_RW_ILV
        hidden_ilv<RES_L0 + li, NS>(
            [&](int j, int kc, int m, const u32x4 (&x)[3], f32x4 acc) {
                const int g = (li * 2 + j) * 4 + kc;
                if (g >= RES_AG) return mfma_bf(t.v[g - RES_AG][wpl(m)], x[xpl(m)], acc);
                const bool first = kc == 0 && m == 0;
                // LAST: the pass's last product, or the one before the VGPR-tail groups (a builtin MFMA then
                // reads the result: srcC forwarding needs no wait, but the compiler may copy it between)
                const bool last = (kc == 3 || g + 1 == RES_AG) && m == 5;
                if (first && last) return mfma_agpr1<true, true>(r.a[g][wpl(m)], x[xpl(m)], acc);
                if (first) return mfma_agpr1<true, false>(r.a[g][wpl(m)], x[xpl(m)], acc);
                if (last) return mfma_agpr1<false, true>(r.a[g][wpl(m)], x[xpl(m)], acc);
                return mfma_agpr1<false, false>(r.a[g][wpl(m)], x[xpl(m)], acc);
            },
            side, lds, wave, lane);
#else
        hidden<RES_L0 + li>(
            [&](int j, int kc, const u32x4 (&x)[3], f32x4 acc) {
                const int g = (li * 2 + j) * 4 + kc;
                if (g < RES_AG) return mfma_x3_agpr(r.a[g][0], r.a[g][1], r.a[g][2], x, acc);
                return mfma_x3(t.v[g - RES_AG], x, acc);
            },
            lds, wave, lane);
#pragma unroll
        for (int k = 0; k < NS; ++k) side(k);
#endif
    }

    // x (4 features) -> fp32 row in XB and the three bf16 planes layer 0 reads
    // split3 (mlp_x3.h) with every remainder through a fence: the same values, no v_pk_add_f32
    static MPCD_DEV void split3s(const f32x4 &v, u32x2 &p0, u32x2 &p1, u32x2 &p2)
    {
        auto fence = [](float &x) { asm volatile("" : "+v"(x)); };
        const uint32_t a = pk_bf16(v.x, v.y), b = pk_bf16(v.z, v.w);
        float r0 = v.x - bf_lo(a), r1 = v.y - bf_hi(a), r2 = v.z - bf_lo(b), r3 = v.w - bf_hi(b);
        fence(r0); fence(r1); fence(r2); fence(r3);
        const uint32_t c = pk_bf16(r0, r1), d = pk_bf16(r2, r3);
        r0 = r0 - bf_lo(c); r1 = r1 - bf_hi(c); r2 = r2 - bf_lo(d); r3 = r3 - bf_hi(d);
        fence(r0); fence(r1); fence(r2); fence(r3);
        p0 = u32x2{a, b};
        p1 = u32x2{c, d};
        p2 = u32x2{pk_bf16(r0, r1), pk_bf16(r2, r3)};
    }

    template <bool FP32 = true>
    static MPCD_DEV void store_x(char *lds, int cl, int n, const f32x4 &x)
    {
        if (FP32) *reinterpret_cast<f32x4 *>(lds + L::XB + (cl * L::SX + n) * 4) = x;
        u32x2 p0, p1, p2;
        split3s(x, p0, p1, p2);
        char *o = lds + L::S1 + cl * L::RS + ((n * 2) ^ (swz(cl) << 4));
        *reinterpret_cast<u32x2 *>(o) = p0;
        *reinterpret_cast<u32x2 *>(o + L::PL) = p1;
        *reinterpret_cast<u32x2 *>(o + 2 * L::PL) = p2;
    }

    using FW = WS<13>;
    // final layer: wave w -> n-tiles w + 4j, both column tiles (a candidate's two CFG rows in one lane); at
    // D0 = 32 and 32 rows load_ws<13>'s SPL mapping (n-tile w & 1) gives waves 0, 1 the same tiles
    static constexpr int NZT = TL<13>;

    // final Linear (32 -> D0) + the denoise update (reference op order, mlp_x3.hip final_and_update)
#ifdef MPCD_PROF_LAYERS
#define MPCD_FINAL_PROF , uint64_t(&tacc)[32]
#define MPCD_FINAL_MARK(k, dep)                                                                                      \
    do {                                                                                                             \
        asm volatile("" ::"v"(dep) : "memory");                                                                     \
        const uint64_t t_ = __builtin_readcyclecounter();                                                            \
        tacc[k] += t_ - tmark;                                                                                       \
        tmark = t_;                                                                                                  \
    } while (0)
#else
#define MPCD_FINAL_PROF
#define MPCD_FINAL_MARK(k, dep)
#endif
    // x_t of the update's (n-tile j, column group g) quads, when MPCD_RW_XREG keeps it in registers
    static constexpr int XG = NB == 2 ? 1 : NCT;
    static MPCD_DEV bool x_lane(int j, int wave, int col)
    {
        return (D0 / 16 % 4 == 0 || wave + 4 * j < D0 / 16) && !(R == 16 && NB == 2 && col >= 8);
    }
    static MPCD_DEV void load_xr(f32x4 (&xr)[NZT][XG], const char *lds, int wave, int lane)
    {
        const int col = lane & 15, q = lane >> 4;
#pragma unroll
        for (int j = 0; j < NZT; ++j)
#pragma unroll
            for (int g = 0; g < XG; ++g) {
                const int cl = NB == 2 ? col : g * 16 + col, n = (wave + 4 * j) * 16 + 4 * q;
                xr[j][g] = x_lane(j, wave, col) ? *reinterpret_cast<const f32x4 *>(lds + L::XB + (cl * L::SX + n) * 4)
                                                : f32x4{0.f, 0.f, 0.f, 0.f};
            }
    }

    static MPCD_DEV void final_and_update(const FW &f, char *lds, const MlpSampleArgs &p, const StepPlan &sp, int s,
                                          int64_t cand0, const f32x4 (&nz)[NZT][NB], uint32_t (&am)[2],
                                          f32x4 (&xr)[NZT][XG], int wave, int lane MPCD_FINAL_PROF)
    {
#ifdef MPCD_PROF_LAYERS
        uint64_t tmark = __builtin_readcyclecounter();
#endif
        constexpr int T = NZT, NT = D0 / 16;
        const int col = lane & 15, q = lane >> 4;
        const float *bias = reinterpret_cast<const float *>(lds + L::BI + A::boff(13) * 4);
        f32x4 acc[T][2];
#pragma unroll
        for (int j = 0; j < T; ++j) {
            const int nt = (NT % 4 == 0 || wave + 4 * j < NT) ? wave + 4 * j : 0;
            acc[j][0] = acc[j][1] = *reinterpret_cast<const f32x4 *>(bias + nt * 16 + 4 * q);
        }
        // both column tiles' operand reads in flight before the first MFMA: one LDS latency instead of two in a row
        u32x4 xf[NCT][3];
#pragma unroll
        for (int c = 0; c < NCT; ++c) load_x3(xf[c], lds + L::T1 + (c * 16 + col) * L::RS + 16 * (q ^ swz(col)), L::PL);
        // MPCD_RW_XREG, DDPM: the x-only products of the update under the operand reads' latency (each through a
        // fence, the same values as in the update's order: a x, c2 x, std z are separate roundings there too)
        constexpr bool PRE = MPCD_RW_XREG && IS_DDPM;
        f32x4 pax[T][XG], pcx[T][XG], psz[T][XG];
        if constexpr (PRE) {
            auto fn = [](float &v) { asm volatile("" : "+v"(v)); };
#pragma unroll
            for (int j = 0; j < T; ++j)
#pragma unroll
                for (int g = 0; g < XG; ++g)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float xv = xr[j][g][r];
                        float a = sp.a * xv, c = sp.c2 * xv, z = sp.std * nz[j][0][r];
                        fn(a); fn(c); fn(z);
                        pax[j][g][r] = a;
                        pcx[j][g][r] = c;
                        psz[j][g][r] = z;
                        am[g] = max(am[g], abs_bits(xv));
                    }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < NCT; ++c)
#pragma unroll
            for (int j = 0; j < T; ++j)
                if (NT % 4 == 0 || wave + 4 * j < NT) acc[j][c] = mfma_x3(f.v[j][0], xf[c], acc[j][c]);
        MPCD_FINAL_MARK(28, acc[0][1]);  // experiment build: the final layer's operand reads and MFMAs
#ifdef MPCD_PROF_FINAL_MFMA_ONLY
        // timing experiment (wrong results): the final layer's MFMAs only, no update
        if (acc[0][0][0] == 12345.f && acc[0][1][1] == 54321.f) am[0] = 1u;
        return;
#endif
        if (R == 16 && NB == 2) {
            // column c holds candidate c & 7's context row (c < 8) or masked row (c >= 8): bring the masked
            // row's eps next to the context row's (DPP row_ror:8 swaps the two halves of each 16-lane row)
#pragma unroll
            for (int j = 0; j < T; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float e = acc[j][0][r];  // element to a scalar first (bit_cast of a vector element)
                    acc[j][1][r] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                        0, __builtin_bit_cast(int, e), 0x128, 0xF, 0xF, false));
                }
            if (col >= 8) return;  // lanes of the masked rows: their eps went to lane col - 8
        }
        const bool last = s == p.n_steps - 1;
#pragma unroll
        for (int j = 0; j < T; ++j) {
            const int nt = wave + 4 * j;
            if (NT % 4 != 0 && nt >= NT) continue;
            const int n = nt * 16 + 4 * q;
#pragma unroll
            for (int g = 0; g < (NB == 2 ? 1 : NCT); ++g) {
                const int cl = NB == 2 ? col : g * 16 + col;
                const f32x4 ec = acc[j][NB == 2 ? 0 : g];
                const f32x4 eu = acc[j][1];
                const int64_t gc = cand0 + cl;
                if (SMODE == MODE_EPS || SMODE == MODE_EPS1) {
                    if (gc < p.batch) {
                        *reinterpret_cast<f32x4 *>(p.x_out + (size_t)gc * D0 + n) = ec;
                        if (SMODE == MODE_EPS) *reinterpret_cast<f32x4 *>(p.chain + (size_t)gc * D0 + n) = eu;
                    }
                    continue;
                }
                const f32x4 x = MPCD_RW_XREG ? xr[j][g] : *reinterpret_cast<const f32x4 *>(lds + L::XB + (cl * L::SX + n) * 4);
                f32x4 xn;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float xv = x[r];
                    float o;
                    if constexpr (PRE) {
                        auto fn = [](float &v) { asm volatile("" : "+v"(v)); };
                        float x0c = pax[j][g][r] - sp.b * ec[r];
                        fn(x0c);
                        float x0u = pax[j][g][r] - sp.b * eu[r];
                        fn(x0u);
                        float x0 = p.wp1 * x0c - p.wf * x0u;
                        x0 = clamp1(x0);
                        float mean = sp.c1 * x0 + pcx[j][g][r];
                        fn(mean);
                        o = (sp.flags & PLAN_NOISE) ? mean + psz[j][g][r] : mean;
                        xn[r] = o;
                        am[g] = max(am[g], abs_bits(o));
                        continue;
                    }
                    if (IS_DDPM) {
                        // every intermediate through a fence: the SLP vectorizer paired the four values' products
                        // into v_pk_mul / v_pk_add_f32, dearer than the plain ops here (same values either way)
                        auto fn = [](float &v) { asm volatile("" : "+v"(v)); };
                        float x0c = sp.a * xv - sp.b * ec[r];
                        fn(x0c);
                        float x0u = sp.a * xv - sp.b * eu[r];
                        fn(x0u);
                        float x0 = p.wp1 * x0c - p.wf * x0u;
                        x0 = clamp1(x0);
                        float mean = sp.c1 * x0 + sp.c2 * xv;
                        fn(mean);
                        o = (sp.flags & PLAN_NOISE) ? mean + sp.std * nz[j][0][r] : mean;
                    } else if (SMODE == MODE_DDIM_CFG) {
                        float x0 = p.wp1 * (sp.a * xv - sp.b * ec[r]) - p.wf * (sp.a * xv - sp.b * eu[r]);
                        if (p.clamp_x0) x0 = clamp1(x0);
                        const float e = p.wp1 * ec[r] - p.wf * eu[r];
                        o = (sp.flags & PLAN_FINAL) ? x0 : x0 * sp.sqan + sp.cn * e;
                    } else {  // MODE_DDIM, 3-arg net
                        float x0 = sp.a * xv - sp.b * ec[r];
                        if (p.clamp_x0) x0 = clamp1(x0);
                        o = (sp.flags & PLAN_FINAL) ? x0 : x0 * sp.sqan + sp.cn * ec[r];
                    }
                    xn[r] = o;
                    am[g] = max(am[g], max(abs_bits(xv), abs_bits(o)));
                }
                store_x<!MPCD_RW_XREG>(lds, cl, n, xn);
                if (MPCD_RW_XREG) xr[j][g] = xn;
                if (gc < p.batch) {
                    if (p.chain) *reinterpret_cast<f32x4 *>(p.chain + ((size_t)(s + 1) * p.batch + gc) * D0 + n) = xn;
                    if (last) *reinterpret_cast<f32x4 *>(p.x_out + (size_t)gc * D0 + n) = xn;
                }
            }
        }
        MPCD_FINAL_MARK(29, am[0]);  // experiment build: the update, the stores
    }

    // noise of step s (slice s+1) for this lane's quads, fetched one step ahead of use
    static MPCD_DEV void fetch_noise(f32x4 (&nz)[NZT][NB], const MlpSampleArgs &p, const StepPlan &sp, int s,
                                     int64_t cand0, int wave, int lane)
    {
        constexpr int NT = D0 / 16;
#pragma unroll
        for (int j = 0; j < NZT; ++j)
#pragma unroll
            for (int g = 0; g < NB; ++g) nz[j][g] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (!IS_DDPM || !(sp.flags & PLAN_NOISE)) return;  // DDIM: sigma = 0
        const int col = lane & 15, q = lane >> 4;
#pragma unroll
        for (int j = 0; j < NZT; ++j) {
            const int nt = wave + 4 * j;
            if (NT % 4 != 0 && nt >= NT) continue;
            const int n = nt * 16 + 4 * q;
            const int64_t gc = cand0 + col;  // DDPM-CFG: NB == 2, one candidate per column (R = 16: columns < 8)
            if (gc >= p.batch || (R == 16 && col >= 8)) continue;
            if (SMODE == MODE_DDPM_XN)
                nz[j][0] = *reinterpret_cast<const f32x4 *>(p.noise + ((size_t)(s + 1) * p.batch + gc) * D0 + n);
            else
                nz[j][0] = philox_normal4(p.seed, (uint64_t)(p.global_offset + gc), (uint32_t)(s + 1), (uint32_t)(n >> 2));
        }
    }

    // The next step's Philox draw (CFG-DDPM with in-kernel noise, one quad per lane) as NPH micro-steps, issued
    // as side work in Linear 8's MFMA slots instead of in the open after Linear 10 (~880 cycles per step there):
    // the exact operations of common.h philox4x32_10 / philox_normal4, one quarter-rate multiply per step,
    // every intermediate through a register fence. Bit-identical to fetch_noise.
    struct PhSt {
        uint32_t c0, c1, c2, c3, k0, k1, h;
        float u0, u1, u2, u3, ra, rb;
        float z[4];
    };
    static constexpr int NPH = 40 + 12;
    static constexpr bool STAGED_NOISE = SMODE == MODE_DDPM_CFG && NZT == 1;
    static MPCD_DEV void ph_init(PhSt &st, const MlpSampleArgs &p, int slice, int64_t cand0, int wave, int lane)
    {
        const int col = lane & 15, q = lane >> 4;
        const int n = min(wave, D0 / 16 - 1) * 16 + 4 * q;  // clamped tile: lanes past NT draw and discard
        const uint64_t cand = (uint64_t)(p.global_offset + cand0 + col);
        st.c0 = (uint32_t)(n >> 2);
        st.c1 = (uint32_t)cand;
        st.c2 = (uint32_t)(cand >> 32);
        st.c3 = (uint32_t)slice;
        st.k0 = (uint32_t)p.seed;
        st.k1 = (uint32_t)(p.seed >> 32);
    }
    static MPCD_DEV void ph_step(PhSt &st, int k)
    {
        auto fu = [](uint32_t &x) { asm volatile("" : "+v"(x)); };
        auto ff = [](float &x) { asm volatile("" : "+v"(x)); };
        constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
        if (k < 40) {  // round k / 4 of philox4x32_10
            switch (k & 3) {
            case 0: st.h = __umulhi(M0, st.c0); fu(st.h); break;                  // hi0
            case 1: st.c0 = M0 * st.c0; fu(st.c0); break;                         // lo0 (in c0 until the swap)
            case 2: { const uint32_t hi1 = __umulhi(M1, st.c2); st.c3 = st.h ^ st.c3 ^ st.k1; st.h = hi1; fu(st.h); fu(st.c3); } break;
            default: {
                const uint32_t lo1 = M1 * st.c2;
                // c' = (hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0); c3 holds hi0 ^ c3 ^ k1, c0 holds lo0
                const uint32_t n0 = st.h ^ st.c1 ^ st.k0, n2 = st.c3, n3 = st.c0;
                st.c0 = n0; st.c1 = lo1; st.c2 = n2; st.c3 = n3;
                st.k0 += W0; st.k1 += W1;
                fu(st.c0); fu(st.c1); fu(st.c2); fu(st.c3);
            } break;
            }
            return;
        }
        const float S = 2.3283064365386963e-10f;  // 2^-32
        switch (k - 40) {  // philox_normal4's Box-Muller
        case 0: st.u0 = ((float)st.c0 + 1.0f) * S; st.u1 = (float)st.c1 * S; ff(st.u0); ff(st.u1); break;
        case 1: st.u2 = ((float)st.c2 + 1.0f) * S; st.u3 = (float)st.c3 * S; ff(st.u2); ff(st.u3); break;
        case 2: st.ra = -2.0f * __logf(st.u0); ff(st.ra); break;
        case 3: st.rb = -2.0f * __logf(st.u2); ff(st.rb); break;
        case 4: st.ra = __fsqrt_rn(st.ra); ff(st.ra); break;
        case 5: st.rb = __fsqrt_rn(st.rb); ff(st.rb); break;
        case 6: st.u1 = 6.2831853071795865f * st.u1; st.u3 = 6.2831853071795865f * st.u3; ff(st.u1); ff(st.u3); break;
        case 7: st.z[0] = __cosf(st.u1); ff(st.z[0]); break;
        case 8: st.z[1] = __sinf(st.u1); ff(st.z[1]); break;
        case 9: st.z[2] = __cosf(st.u3); ff(st.z[2]); break;
        case 10: st.z[3] = __sinf(st.u3); ff(st.z[3]); break;
        default:
            for (int e = 0; e < 4; ++e) {
                st.z[e] = (e < 2 ? st.ra : st.rb) * st.z[e];
                ff(st.z[e]);
            }
            break;
        }
    }
    // fetch_noise's result from the staged draw: zeros where fetch_noise draws none
    static MPCD_DEV void ph_take(f32x4 (&nz)[NZT][NB], const PhSt &st, const StepPlan &sp, int64_t cand0,
                                 const MlpSampleArgs &p, int wave, int lane)
    {
        const int col = lane & 15;
#pragma unroll
        for (int g = 0; g < NB; ++g) nz[0][g] = f32x4{0.f, 0.f, 0.f, 0.f};
        const bool ok = (sp.flags & PLAN_NOISE) && (D0 / 16 % 4 == 0 || wave < D0 / 16) && cand0 + col < p.batch &&
                        !(R == 16 && col >= 8);
        if (ok) nz[0][0] = f32x4{st.z[0], st.z[1], st.z[2], st.z[3]};
    }

    static MPCD_DEV void run(const MlpSampleArgs &p)
    {
        extern __shared__ float lds_f[];
        char *lds = reinterpret_cast<char *>(lds_f);
        const int lane = threadIdx.x & 63;
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const int64_t cand0 = (int64_t)blockIdx.x * CPW;
        int lane16 = lane * 16;
        const float *wp = p.wpack;
        float *bi = reinterpret_cast<float *>(lds + L::BI);
        float *bic = reinterpret_cast<float *>(lds + L::BIC);
        float *cps = reinterpret_cast<float *>(lds + L::CPS);

#if MPCD_RW_EXP_NOLASTEPI
        // the timing experiment leaves output tiles unwritten: start from a zeroed LDS so they read finite values
        for (int i = threadIdx.x; i < L::total / 16; i += RW_T) reinterpret_cast<u32x4 *>(lds)[i] = u32x4{0u, 0u, 0u, 0u};
        lds_barrier();
#endif
        Res res;
        load_res(res, wp, wave, lane);
        for (int l = 0; l < NLAYER; ++l)
            for (int i = threadIdx.x; i < A::N[l]; i += RW_T) bi[A::boff(l) + i] = wp[woffx<D0>(l) + wfl<D0>(l) + i];
        for (int j = 0; j < 6; ++j)
            for (int i = threadIdx.x; i < A::N[2 * j + 1]; i += RW_T)
                bic[cond_off(j) + i] = wp[woffx<D0>(2 * j + 1) + wfl<D0>(2 * j + 1) + i];
        // mpcd_mpc_step (ctx_fused): the shared context row's projection computed here, as ctx_prologue_row_kernel
        // would (the same function: the same bits), so the control step has no prologue launch
        for (int i = threadIdx.x; i < COND_TOTAL; i += RW_T)
            cps[i] = !CTX ? 0.f
                          : p.ctx_fused ? ctx_proj_col(p.ctx_row, p.ctx_dim, p.cond_layers, p.n_cond, p.cond_dim, i)
                                        : p.cproj[i];
        if (threadIdx.x < CPW) reinterpret_cast<uint32_t *>(lds + L::AMX)[threadIdx.x] = 0u;
        uint32_t am[2] = {0u, 0u};
        for (int i = threadIdx.x; i < CPW * QUADS; i += RW_T) {  // x_T (fp32 + planes)
            const int c = i / QUADS, qd = i - c * QUADS;
            const int64_t gc = cand0 + c;
            f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
            if (gc < p.batch) {
                z = p.noise ? *reinterpret_cast<const f32x4 *>(p.noise + (size_t)gc * D0 + qd * 4)
                            : philox_normal4(p.seed, (uint64_t)(p.global_offset + gc), 0u, (uint32_t)qd);
                if (p.chain && SMODE != MODE_EPS) *reinterpret_cast<f32x4 *>(p.chain + (size_t)gc * D0 + qd * 4) = z;
            }
            store_x(lds, c, qd * 4, z);
        }
        f32x4 xr[NZT][XG];
        if constexpr (MPCD_RW_XREG) {
            lds_barrier();
            load_xr(xr, lds, wave, lane);
        }

        int wofs = 0;
        WS<0> w0;
        load_ws<0>(w0, wp, wave, lane16);
        f32x4 nz[NZT][NB];
        StepPlan sp = load_plan(p.plan, 0);
        fetch_noise(nz, p, sp, 0, cand0, wave, lane);
        const int tpi = threadIdx.x < COND_TOTAL / 4 ? (int)threadIdx.x : threadIdx.x < COND_TOTAL / 2 ? (int)threadIdx.x - COND_TOTAL / 4 : 0;
        f32x4 tpre = reinterpret_cast<const f32x4 *>(p.tproj)[tpi];
#ifdef MPCD_PROF_LAYERS
        // experiment build only: per-wave shader-clock cycles of each segment (work, then barrier wait), the
        // dump format of mlp_x3.hip (tools/layer_prof.py)
        uint64_t tacc[2 * 16] = {};
        const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
        uint64_t tprev = __builtin_readcyclecounter();
        const uint64_t ct0 = tprev;
        int bk = 0;
        auto bar = [&] {
            uint64_t t = __builtin_readcyclecounter();
            tacc[2 * bk] += t - tprev;
            lds_barrier();
            tprev = __builtin_readcyclecounter();
            tacc[2 * bk + 1] += tprev - t;
            bk = bk == 13 ? 0 : bk + 1;
        };
#else
#if MPCD_RW_EXP_BAR2
        auto bar = [] { lds_barrier(); lds_barrier(); };  // timing experiment: the cost of one more barrier per layer
#else
        auto bar = [] { lds_barrier(); };
#endif
#endif

        for (int s = 0; s < p.n_steps; ++s) {
            // launder the weight base: stops LICM hoisting the streamed layers' loads out of the loop
            asm volatile("" : "+s"(wofs), "+v"(lane16));
            const float *ws = wp + wofs;
            auto none = [](int) {};
            // Each layer's fragments are issued one at a time in the free MFMA slots of an earlier layer
            // (hidden_ilv side work): the vector-memory issue rides under MFMAs instead of stalling a layer, and
            // the register budget (one wave per SIMD, 512 registers, 252 AGPRs of resident weights) holds: L8's
            // 96 registers are in flight from L5 on, everything else one or two layers ahead.
            WS<1> w1;
            load_ws<1>(w1, ws, wave, lane16);
            WS<2> w2;
            load_ws<2>(w2, ws, wave, lane16);
            bar();
            // this step's time projections + cond biases (+ shared context part) -> TPU / TPC: one f32x4 per thread
            auto table = [&] {
                if (threadIdx.x < COND_TOTAL / 2) {
                    const bool ctx_half = threadIdx.x >= COND_TOTAL / 4;
                    const int k = ctx_half ? (int)threadIdx.x - COND_TOTAL / 4 : (int)threadIdx.x;
                    f32x4 u = tpre + reinterpret_cast<const f32x4 *>(lds + L::BIC)[k];
                    if (ctx_half) u = u + reinterpret_cast<const f32x4 *>(lds + L::CPS)[k];
                    reinterpret_cast<f32x4 *>(lds + (ctx_half ? L::TPC : L::TPU))[k] = u;
                }
            };
            if (!MPCD_RW_TABLE_EARLY || s == 0) {
                table();
                tpre = reinterpret_cast<const f32x4 *>(p.tproj + (size_t)(s + 1 < p.n_steps ? s + 1 : s) * COND_TOTAL)[tpi];
            }
            WS<3> w3;
            layer<0, NFRAG<3>>(w0, [&](int k) { load_ws1<3>(w3, ws, wave, lane16, k); }, lds, wave, lane);
            bar();
            WS<4> w4;
            WS<8> w8;
            Tail tail;
            WS<9> w9;
            WS<10> w10;
            WS<11> w11;
            WS<12> w12;
            WS<13> w13;
            const StepPlan cur = sp;
            PhSt ph;
            auto side9 = [&](int k) {
                if (k < NFRAG<11>) load_ws1<11>(w11, ws, wave, lane16, k);
                else if (k < NFRAG<11> + NFRAG<12>) load_ws1<12>(w12, ws, wave, lane16, k - NFRAG<11>);
                else load_ws1<13>(w13, ws, wave, lane16, k - NFRAG<11> - NFRAG<12>);
            };
            f32x4 nzc[NZT][NB];
            auto noise_next = [&] {  // this step's noise to nzc, the next step's drawn / fetched into nz
#pragma unroll
                for (int j = 0; j < NZT; ++j)
#pragma unroll
                    for (int g = 0; g < NB; ++g) nzc[j][g] = nz[j][g];
                if (STAGED_NOISE && s + 1 < p.n_steps) {
                    ph_take(nz, ph, sp, cand0, p, wave, lane);
                } else if (s + 1 < p.n_steps) {
#ifdef MPCD_PROF_LAYERS
                    const uint64_t tn0 = __builtin_readcyclecounter();
#endif
                    fetch_noise(nz, p, sp, s + 1, cand0, wave, lane);
#ifdef MPCD_PROF_LAYERS
                    asm volatile("" ::: "memory");
                    tacc[31] += __builtin_readcyclecounter() - tn0;  // "tail" row, wait column: the noise draws
#endif
                }
            };
            layer<1, NFRAG<4>>(w1, [&](int k) { load_ws1<4>(w4, ws, wave, lane16, k); }, lds, wave, lane);
            bar();
            layer<2>(w2, none, lds, wave, lane);
            bar();
            layer<3>(w3, none, lds, wave, lane);
            bar();
            layer<4>(w4, none, lds, wave, lane);
            bar();
            constexpr int W8A = MPCD_RW_W8_SPLIT ? NFRAG<8> / 2 : 0;  // Linear 8 fragments issued during Linear 5
            layer_res<0, W8A>(res, tail, [&](int k) { load_ws1<8>(w8, ws, wave, lane16, k); }, lds, wave, lane);
            bar();
            layer_res<1, NFRAG<8> - W8A>(res, tail, [&](int k) { load_ws1<8>(w8, ws, wave, lane16, W8A + k); }, lds, wave,
                                         lane);
            load_tail(tail, ws, wave, lane16);
            bar();
            layer_res<2>(res, tail, none, lds, wave, lane);
            load_ws<9>(w9, ws, wave, lane16);
            bar();
            if (s + 1 < p.n_steps) sp = load_plan(p.plan, s + 1);
            if constexpr (STAGED_NOISE) {
                ph_init(ph, p, s + 2, cand0, wave, lane);  // step s + 1's noise is Philox slice s + 2 (fetch_noise)
                layer<8, NPH>(w8, [&](int k) { ph_step(ph, k); }, lds, wave, lane);
            } else {
                layer<8>(w8, none, lds, wave, lane);
            }
            load_ws<10>(w10, ws, wave, lane16);  // after L8: w8's 96 registers are free again
            bar();
            layer<9, NFRAG<11> + NFRAG<12> + NFRAG<13>>(w9, side9, lds, wave, lane);
            bar();
            layer<10>(w10, none, lds, wave, lane);
            noise_next();
            load_ws<0>(w0, ws, wave, lane16);  // next step's layer 0 (unconditional: path-independent load count)
            bar();
            layer<11>(w11, none, lds, wave, lane);
            bar();
            if constexpr (MPCD_RW_TABLE_EARLY && MPCD_RW_TABLE_SIDE) {
                // step s + 1's tables as Linear 12's side work: both reads in its first MFMA slot, the add and the
                // write in its last (Linear 11 read step s's tables last; the barrier above orders them)
                constexpr int NS12 = TL<12> * CL<12> * (A::K[12] / 32) * 6;
                const bool ctx_half = threadIdx.x >= COND_TOTAL / 4;
                f32x4 tb0, tb1;
                layer<12, NS12>(w12, [&](int k) {
                    if (k == 0) {
                        tb0 = reinterpret_cast<const f32x4 *>(lds + L::BIC)[tpi];
                        tb1 = reinterpret_cast<const f32x4 *>(lds + L::CPS)[tpi];
                    } else if (k == NS12 - 1 && s + 1 < p.n_steps && threadIdx.x < COND_TOTAL / 2) {
                        f32x4 u = tpre + tb0;
                        if (ctx_half) u = u + tb1;
                        reinterpret_cast<f32x4 *>(lds + (ctx_half ? L::TPC : L::TPU))[tpi] = u;
                    }
                }, lds, wave, lane);
                if (s + 1 < p.n_steps)
                    tpre = reinterpret_cast<const f32x4 *>(p.tproj + (size_t)(s + 2 < p.n_steps ? s + 2 : s + 1) * COND_TOTAL)[tpi];
            } else {
                if (MPCD_RW_TABLE_EARLY && s + 1 < p.n_steps) {  // step s + 1's tables (Linear 11 read step s's last)
                    table();
                    tpre = reinterpret_cast<const f32x4 *>(p.tproj + (size_t)(s + 2 < p.n_steps ? s + 2 : s + 1) * COND_TOTAL)[tpi];
                }
                layer<12>(w12, none, lds, wave, lane);
            }
            bar();
#ifdef MPCD_PROF_LAYERS
            final_and_update(w13, lds, p, cur, s, cand0, nzc, am, xr, wave, lane, tacc);  // "-" row: MFMAs / update
#else
            final_and_update(w13, lds, p, cur, s, cand0, nzc, am, xr, wave, lane);
#endif
        }
#ifdef MPCD_PROF_LAYERS
        {
            const uint64_t t = __builtin_readcyclecounter();
            tacc[2 * 15] += t - tprev;
            if (p.dbg && blockIdx.x < 32 / RW_W && lane == 0)  // 32 wave slots
                for (int i = 0; i < 32; ++i) p.dbg[(blockIdx.x * RW_W + (threadIdx.x >> 6)) * 32 + i] = (float)tacc[i];
            if (p.dbg && threadIdx.x == 0) {  // per-block loop start / end (memrealtime, low 32 bits)
                p.dbg[4096 + blockIdx.x * 2] = __builtin_bit_cast(float, (uint32_t)rt0);
                p.dbg[4096 + blockIdx.x * 2 + 1] = __builtin_bit_cast(float, (uint32_t)__builtin_amdgcn_s_memrealtime());
            }
            if (p.dbg && blockIdx.x < 8 && threadIdx.x == 0) {  // shader clock = d(memtime) / d(memrealtime) x 100 MHz
                p.dbg[8 * 4 * 32 + blockIdx.x * 2] = (float)(t - ct0);
                p.dbg[8 * 4 * 32 + blockIdx.x * 2 + 1] = (float)(__builtin_amdgcn_s_memrealtime() - rt0);
            }
        }
#endif
        if (SMODE != MODE_EPS && SMODE != MODE_EPS1 && p.chain_absmax) {
            const int col = lane & 15;
            store_chain_absmax<CPW, RW_T>(reinterpret_cast<uint32_t *>(lds + L::AMX), am, col,
                                          (NB == 2 || R == 16) ? -1 : 16 + col, NB == 1 || R == 32 || col < 8,
                                          p.chain_absmax, cand0, p.batch);
        }
    }
};

template <int D0, int SMODE, bool CTX, int R>
__global__ __launch_bounds__(RW_T, 1) void mlp_rw_kernel(const MlpSampleArgs p)
{
    MlpRw<D0, SMODE, CTX, R>::run(p);
}

template <int D0, int SMODE, bool CTX, int R>
hipError_t launch_rw_r(const MlpSampleArgs &a, hipStream_t stream)
{
    using L = Lds3<D0, MlpRw<D0, SMODE, CTX, R>::NB, R>;
    static_assert(L::total <= 160 * 1024, "LDS budget (160 KiB per CU)");
    if (hipError_t e = allow_max_lds<&mlp_rw_kernel<D0, SMODE, CTX, R>>(); e != hipSuccess) return e;
    const int64_t blocks = (a.batch + L::CPW - 1) / L::CPW;
    return launch_sampler_kernel(mlp_rw_kernel<D0, SMODE, CTX, R>, dim3((unsigned)blocks), dim3(RW_T), (size_t)L::total, stream, a);
}

template <int D0, int SMODE, bool CTX>
hipError_t launch_rw(const MlpSampleArgs &a, int rows, hipStream_t stream)
{
    return rows == 16 ? launch_rw_r<D0, SMODE, CTX, 16>(a, stream) : launch_rw_r<D0, SMODE, CTX, 32>(a, stream);
}

template <int D0>
hipError_t launch_rw_d0(const MlpSampleArgs &a, int rows, hipStream_t stream)
{
    const bool ctx = a.cproj != nullptr;
    switch (a.mode) {
    case MODE_DDPM_CFG:
        if (a.noise) return ctx ? launch_rw<D0, MODE_DDPM_XN, true>(a, rows, stream) : launch_rw<D0, MODE_DDPM_XN, false>(a, rows, stream);
        return ctx ? launch_rw<D0, MODE_DDPM_CFG, true>(a, rows, stream) : launch_rw<D0, MODE_DDPM_CFG, false>(a, rows, stream);
    case MODE_DDIM_CFG: return ctx ? launch_rw<D0, MODE_DDIM_CFG, true>(a, rows, stream) : launch_rw<D0, MODE_DDIM_CFG, false>(a, rows, stream);
    case MODE_DDIM: return ctx ? launch_rw<D0, MODE_DDIM, true>(a, rows, stream) : launch_rw<D0, MODE_DDIM, false>(a, rows, stream);
    case MODE_EPS: return ctx ? launch_rw<D0, MODE_EPS, true>(a, rows, stream) : launch_rw<D0, MODE_EPS, false>(a, rows, stream);
    case MODE_EPS1: return ctx ? launch_rw<D0, MODE_EPS1, true>(a, rows, stream) : launch_rw<D0, MODE_EPS1, false>(a, rows, stream);
    }
    return hipErrorInvalidValue;
}

}  // namespace

// rows: 32 or 16 per workgroup (mlp_x3.hip picks, as for its own layouts)
hipError_t launch_mlp_rw(int d0, int rows, const MlpSampleArgs &a, hipStream_t stream)
{
    switch (d0) {
    case 32: return launch_rw_d0<32>(a, rows, stream);
    case 64: return launch_rw_d0<64>(a, rows, stream);
    case 128: return launch_rw_d0<128>(a, rows, stream);
    }
    return hipErrorInvalidValue;
}
