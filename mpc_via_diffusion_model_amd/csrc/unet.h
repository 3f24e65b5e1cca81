// 1D temporal U-Net sampler (ConditionedTemporalUnet / TemporalUnet) — internal interface.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "../../include/mpcd.h"
#include "internal.h"

// One fused conv launch of the U-Net (see unet.hip for the op list).
struct ConvLayer {
    int kind;          // CONV_SAME5 / CONV_DOWN3 / CONV_UP4 / CONV_PW1
    int cin, cout;     // total input channels (a + b concat), output channels
    int coutp;         // cout padded to a multiple of 16 (MFMA n-tiles)
    int cinp;          // cin padded to a multiple of 4 (first layer: d -> 4/8)
    int kpad;          // packed K per parity, multiple of 16
    const float *w;    // packed A operand (device), [parities][cout/16][kpad/16][64][4]
    const float *bias; // [cout]
    const float *gn_w, *gn_b;  // GroupNorm affine or null
    int groups;
    int cond_off;      // column of this block in tproj/cproj, -1 = none
    // bf16 / f16 MFMA form (MPCD_F32X3, MPCD_F16; unet_mx.hip): [parities][coutp/16][kc][planes][64][8]
    const uint16_t *wmx;
    int cinp8;         // cin padded to 8 / 16 / a multiple of 32 (K per tap)
    int kc;            // k-chunks of 32 per parity
    // two-term fp16 form (MPCD_F16X2; the fused U-Net): [parities][coutp/16][kc][2][64][8] of the weights x 1/inv2
    const uint16_t *wmx2;
    float inv2;        // 1 / the conv's power-of-two weight scale
};

// One fused conv launch of the bf16/f16-MFMA family (unet_mx.hip).
struct ConvMK {
    const float *xa, *xb;   // inputs [x_rows][lin][ca], [x_rows][lin][cb] (channel concat)
    int ca, cb, cinp, kc;   // channels, padded channels per tap, k-chunks of 32
    int64_t x_rows;         // row r reads input row r % x_rows
    const uint16_t *w;      // packed A fragments
    const float *bias;
    const float *gn_w, *gn_b;
    int groups;
    const float *tp, *cp;   // cond (EPI_GN_MISH_COND): tproj row + cond_off, cproj + cond_off or null
    int64_t cp_stride, b_cand;
    const float *res;       // residual [rows][lout][cout] (EPI_GN_MISH_RES)
    float *out;             // [rows][lout][cout]
    int64_t rows;
    int lin, lout, cout, coutp;
    int rb;                 // rows per workgroup
    int halo_l, halo_r;     // staged input window = [-halo_l, lin + halo_r)
    int cs;                 // staged bytes per position (one plane)
    int epi;                // EPI_*
    int alias;              // 1: the fp32 output tile reuses the staged-input LDS
    int stat_off;           // LDS byte offset of the GroupNorm statistics (then the per-channel table)
    int cpg_shift;          // log2(cout / groups)
    int skip;               // experiment only (MPCD_UNET_SKIP): bit 0 staging, 1 GEMM, 2 statistics, 3 epilogue
    // LDS placement (set by unet_launch_mx / unet_launch_mx_rtb): staged input planes and fp32 tile
    int in_off, out_off;
    // fused ResidualTemporalBlock, first conv only: the epilogue writes its result as the second
    // conv's staged planes (LDS offset nx_off, per-position stride nx_cs, window nx_win, left halo
    // nx_halo_l) instead of storing it to HBM
    int lds_out, nx_off, nx_cs, nx_win, nx_halo_l;
    // fp16 activation buffers (f16 net): input (xa / xb), residual, output hold halves, not floats
    int in_h, res_h, out_h;
    int layer;              // index of the conv in UnetWeights::layers (diagnostics)
    // first-generation stagger (non-persistent grids): workgroup b < stag_ncu * stag_slots sleeps
    // (b / stag_ncu) * stag_units x s_sleep(32), so the co-resident workgroups of a CU run their
    // staging / GEMM / epilogue phases out of step instead of all at once
    int stag_units, stag_ncu, stag_slots;
    uint32_t *wgtrace;      // diagnostics (MPCD_UNET_WGTRACE): per workgroup {start, end, HW_ID, XCC_ID}
};

// Whole-network-per-workgroup form (unet_fused.hip): the op program and its LDS placement.
struct UnetFusedPlan;
void unet_fused_free(UnetFusedPlan *p);

struct UnetWeights {
    bool ready = false;
    int n_layers = 0;
    int planes = 0;                 // 0: fp32 MFMA kernels (unet.hip); 3: split-bf16, 1: f16 (unet_mx.hip)
    int fused_planes = 0;           // the fused program's numerics when they differ from planes (2: MPCD_F16X2)
    std::vector<ConvLayer> layers;  // in execution order (see unet.hip build_plan)
    std::shared_ptr<UnetFusedPlan> fused;  // null when the fused form does not cover the net
    std::shared_ptr<UnetFusedPlan> fused3; // MPCD_F16X2 nets: the split-bf16 fused program, for the unclamped DDIM
                                           // samplers (their x leaves the fp16 range)
    std::string fused_why;                 // why not (diagnostics)
    bool force3 = false;                   // mpcd_force_f32x3: an MPCD_F16X2 net runs its split-bf16 program everywhere
};

struct UnetSampleArgs {
    const StepPlan *plan;
    const StepPlan *plan_host;
    const float *tproj;
    const float *cproj;
    int64_t cproj_stride;
    int32_t cond_total;
    const float *noise;
    float *x_out;
    float *chain;
    float *chain_absmax;           // [B] or null: max |x| over the chain per candidate (mpcd_sample_args)
    int64_t batch;
    int64_t global_offset;
    uint64_t seed;
    int32_t n_steps;
    int32_t mode;
    int32_t clamp_x0;
    float wp1, wf;
    void *workspace;
    float *eps_cond, *eps_uncond;  // MODE_EPS / MODE_EPS1 outputs
    const float *x_in;             // MODE_EPS / MODE_EPS1 input
    int32_t fused;                 // the form, decided once per call by unet_use_fused (it also sized workspace)
};

// epilogue kinds shared by both conv families
enum { UCONV_SAME5 = 0, UCONV_DOWN3 = 1, UCONV_UP4 = 2, UCONV_PW1 = 3 };
enum { UEPI_BIAS = 0, UEPI_GN_MISH = 1, UEPI_GN_MISH_COND = 2, UEPI_GN_MISH_RES = 3 };

// Pack one conv for the MFMA-bf16/f16 kernels; planes = 3 (split-bf16, MPCD_F32X3) or 1 (f16, MPCD_F16).
// w_host: conv [cout][cin][ks] or convT [cin][cout][4]. Appends to `pack` and sets L.wmx (offset), L.cinp8, L.kc.
// planes 1 (fp16), 3 (split bf16) -> L.wmx; 2 (two-term fp16 of the weights x scale) -> L.wmx2, L.inv2 = 1 / scale
void unet_pack_mx(int kind, int cin, int cout, int planes, const float *w_host, ConvLayer &L,
                  std::vector<uint16_t> &pack);
// Choose rows per workgroup / tile shape and launch; kind = UCONV_*, planes 1 or 3.
hipError_t unet_launch_mx(int kind, int planes, ConvMK &k, hipStream_t st, std::string *why);

// A ResidualTemporalBlock's two 5-tap convs (k1: conv1 + GN/Mish/cond -> k1.out; k2: conv2 + GN/Mish
// + residual, k2.xa = k1.out) as one fused launch when that measures faster than the pair (the
// intermediate then stays in LDS and k1.out is not written). MPCD_UNET_FUSE=0/1 forces either form.
hipError_t unet_launch_mx_rtb(int planes, ConvMK &k1, ConvMK &k2, hipStream_t st, std::string *why);

// One denoise step of the fused form (unet_fused_step): x [B][H][d] is updated in place (or is the input of
// MODE_EPS, whose eps of both branches go to eps_c / eps_u).
struct UnetFusedStep {
    float *x;
    int64_t batch, goff;
    int mode, clamp_x0, step, last;
    const float *tp, *cp;  // tproj row of this step, cproj (or null)
    int64_t cp_stride;
    const StepPlan *plan;
    float wp1, wf;
    const float *noise;
    uint64_t seed;
    float *chain, *x_out;
    uint32_t *amq;
    float *eps_c, *eps_u;
    void *scratch;  // unet_fused_scratch_bytes
    uint64_t *prof;  // diagnostics: [unet_fused_prof_wgs()][n_ops][4] s_memtime stamps, or null
};
// planes: the program's numerics (0: the net's own - W.fused_planes, else W.planes; 3: the split-bf16 program of an
// MPCD_F16X2 net)
UnetFusedPlan *unet_fused_prepare(const mpcd_net_desc &d, const UnetWeights &W, int rows_per_wg, std::string *why,
                                  int planes = 0);
size_t unet_fused_scratch_bytes(const UnetFusedPlan &pl, int64_t batch);
// true: the fused launch writes each branch's eps (one row per workgroup) and the CFG update runs as its own launch
bool unet_fused_split_update(const UnetFusedPlan &pl);
int unet_fused_rows_per_wg(const UnetFusedPlan &pl);
int unet_fused_planes(const UnetFusedPlan &pl);
int unet_fused_n_ops(const UnetFusedPlan &pl);
int unet_fused_prof_wgs();
// kind, epi, cinp, cout, lout, k-chunks, n-tiles per wave, column tiles per wave
void unet_fused_op_info(const UnetFusedPlan &pl, int i, int32_t out[8]);
hipError_t unet_fused_step(const UnetFusedPlan &pl, const UnetFusedStep &s, hipStream_t st);
// mpcd_unet_force_path: 0 = automatic, 1 = layer by layer, 2 = fused (error where it does not apply)
void unet_force_path(int path);
// the form a sample call of sampler `mode` takes: out = {1 fused / 0 layer by layer, operand planes (0 = fp32
// FMA, 1 = fp16, 3 = split bf16), rows and waves per workgroup of the fused program (0 when layered)}
void unet_form(const UnetWeights &W, int mode, int32_t out[4]);
int unet_fused_waves_per_wg(const UnetFusedPlan &pl);

// mpcd_unet_force_tiling (include/mpcd.h)
void unet_force_tiling(int conv, int block);

using TensorLookup = std::function<const float *(const char *)>;

// dev(name): device pointer of a blob tensor; host(name): host pointer of the same tensor.
// Repacks conv weights into `pack` (device, grown as needed).
int unet_prepare(const mpcd_net_desc &d, size_t n_tensors, const TensorLookup &dev, const TensorLookup &host,
                 UnetWeights &w, void *&pack, size_t &pack_bytes);
// Whole-net (fused) or layer-by-layer form of one sample / eps call: read once per call (the process-wide
// override may change between calls, from any thread) and passed to both the workspace sizing and the call.
bool unet_use_fused(const UnetWeights &w, int mode);
size_t unet_workspace_bytes(const mpcd_net_desc &d, const UnetWeights &w, bool fused, int64_t batch, int nb);
int unet_sample(const mpcd_net_desc &d, const UnetWeights &w, const UnetSampleArgs &a, hipStream_t stream);
const char *unet_last_error();
