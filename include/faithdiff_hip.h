/*
 * faithdiff_hip.h -- C ABI of libfaithdiff_hip.so, the MI355X (gfx950) device path of the
 * FaithDiff denoising hot path.
 *
 * The reference (tpetkovich/FaithDiff-dev) owns no native code: every op below replaces an
 * *implicit* ATen kernel that diffusers 0.28 / torch 2.4 launch for it.  The
 * reference call site each entry point replaces is cited next to it.
 *
 * Conventions
 *   - Activations are NHWC ("[M, C]" row-major with M = batch*H*W); weights row-major [N][K].
 *   - dtype codes: FD_BF16 (UNet), FD_F16 (VAE / denoise encoder), FD_F32.
 *   - Every function returns 0 (FD_OK) or a negative fd_status; the Python layer raises
 *     RuntimeError on non-zero.  No allocation and no host synchronisation happens inside an op,
 *     so every op is capturable into a hipGraph.  Caller owns every buffer.
 *   - `stream` is a hipStream_t (NULL = legacy default stream).
 */
#ifndef FAITHDIFF_HIP_H
#define FAITHDIFF_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  FD_OK = 0,
  FD_ERR_SHAPE = -1,   /* unsupported / inconsistent shape */
  FD_ERR_DTYPE = -2,   /* unsupported dtype combination */
  FD_ERR_ARCH = -3,    /* device is not gfx950 */
  FD_ERR_HIP = -4,     /* a HIP runtime call failed (launch error) */
  FD_ERR_ARG = -5      /* null pointer / bad argument */
} fd_status;

enum { FD_BF16 = 0, FD_F16 = 1, FD_F32 = 2 };
enum { FD_ACT_NONE = 0, FD_ACT_SILU = 1, FD_ACT_GELU = 2, FD_ACT_QUICKGELU = 3, FD_ACT_GEGLU = 4, FD_ACT_LRELU = 5,
       FD_ACT_SOFTMAX = 6 };

/* ---------------------------------------------------------------------------------------------
 * GEMM / implicit-GEMM convolution on MFMA (v_mfma_f32_16x16x32_{bf16,f16}), operands staged through
 * LDS by global_load_lds.  Two kernels: 8-wave 256-row tiles with in-launch split-K (M >= 256) and
 * 4-wave 128/64-row tiles (small M, batched).  C[b][m][n] = epi( alpha * sum_k A[b][m][k] * B[b][n][k] ).
 *   epi(v) = act(v + bias[n] + rowbias[(m / rows_per_group) * rowbias_ld + n]) + residual[m][n]
 *   act == FD_ACT_GEGLU: B rows are packed in groups of 32 = [16 "hidden" | 16 "gate"]; the
 *   output has N/2 columns: out = (h + b_h) * gelu(g + b_g)   (diffusers GEGLU).
 * conv != 0 turns A into an implicit im2col gather from an NHWC image (K = 9*Cin, tap-major):
 *   3x3 kernel, stride 1|2, symmetric pad `pad` (bottom/right zero-fill handles the VAE's
 *   (0,1,0,1) pad with pad = 0), optional nearest upsample folded into the gather (Upsample2D:
 *   upsample=1 resizes Hin x Win -> Hout x Wout with src = dst*in/out, i.e. x2 or diffusers'
 *   upsample_size for latents that are not multiples of 4; needs stride 1, pad 1), optional channel concat of two sources (A: C1 channels, A2: Cin-C1 channels).
 * Replaces: cuBLAS addmm/mm behind every nn.Linear and cuDNN conv2d behind every nn.Conv2d of
 *   ResnetBlock2D / Transformer2DModel / Down-/Upsample2D (diffusers; called from
 *   unet_2d_condition_vae_extension.py:571-690 and pipeline_FaithDiff_tlc.py:970,1272,1438).
 * Requires K % 64 == 0 (and Cin % 64 == 0, C1 % 64 == 0 for conv).
 * ------------------------------------------------------------------------------------------- */
typedef struct fd_gemm_params {
  const void* A;
  const void* B;
  void* C;
  long long lda, ldb, ldc;
  long long strideA, strideB, strideC;
  int M, N, K, batch;
  const float* bias;
  const void* residual;
  long long ldr, strideR;
  const float* rowbias;
  long long rowbias_ld;
  int rows_per_group;
  float alpha;
  int act;
  int dtype;
  int out_dtype;
  /* implicit-GEMM conv */
  int conv;
  int nimg, Hin, Win, Cin, Hout, Wout, stride, pad, upsample;
  const void* A2;
  int C1;
  /* split-K / tiling (0 / NULL = defaults).  m_ref: rows of ONE TLC tile's forward; the split-K count
   * (the only choice that changes summation order) is derived from (m_ref, N, K), so batching tiles
   * into one launch leaves every output bit unchanged.  ws: caller-owned workspace of at least
   * fd_gemm_ws_bytes(p) bytes whose first 256 KiB (split-K tile counters) are zero before the first
   * launch; launches leave them zero again. */
  int m_ref;
  void* ws;
  long long ws_bytes;
  /* LayerNorm folded across a GEMM pair (Transformer blocks' norm1/2/3, diffusers BasicTransformerBlock;
   * replaces the separate LayerNorm launch).  Producer (ln_out != NULL; N % 160 == 0, no GEGLU, batch 1):
   * also writes, per output row m and 160-column group g, (sum, sum of squares) of the STORED outputs
   * to ln_out[m * (N / 160) + g] (float2).  Consumer (ln_in != NULL; K % 320 == 0, K <= 1280, batch 1):
   * A is the producer's raw output x; B holds W' = W * gamma (per k), ln_c[n] = sum_k W'[n][k], bias =
   * W . beta + b; the epilogue computes rstd_m * (acc - mean_m * ln_c[n]) + bias[n] = LN(x) . W^T + b with
   * (mean_m, rstd_m) from the producer's partials (eps ln_eps), before the activation / GEGLU. */
  float* ln_out;
  const float* ln_in;
  const float* ln_c;
  float ln_eps;
  /* GroupNorm statistics of the output for the GroupNorm that consumes it (VAE / UNet resnets: conv2 -> next
   * norm1, conv1 -> norm2; replaces the gn_partial pass of fd_group_norm).  Request: gn_part != NULL,
   * gn_groups = G, gn_hw = rows per image.  When the chosen kernel can produce them (256-row tiles of gemm8 /
   * gemm256, or the 128 x 128 tiles of the 4-wave kernel; every tile inside one image: gn_hw % R == 0, its
   * columns a whole number of groups, the vector epilogue; no GEGLU / LayerNorm fold) fd_gemm writes, per image i,
   * R-row block b and group g, (sum, sum of squares) of the STORED outputs to gn_part[(i * gn_hw / R + b) * G + g]
   * (float2) and sets gn_done = R (256 or 128), else 0 (then the consumer runs the full fd_group_norm).  Size
   * gn_part for R = 128.  Consumer: fd_group_norm_partials(..., part_rows = gn_done, ...). */
  float* gn_part;
  int gn_groups;
  int gn_hw;
  int gn_done;
  /* Consumer GroupNorm (+ SiLU) folded into a 3x3 stride-1 conv (the halo-staged kernel only: callers check
   * fd_conv_halo_plan first; an ineligible conv with gi_affine set returns FD_ERR_SHAPE).  gi_affine: fp32
   * (scale, shift) per (image, input channel), [nimg][Cin][2], from fd_group_norm_affine, with 64 channels of
   * padding after the last image; the conv reads silu?(x * scale + shift) rounded to the input type, zero outside
   * the image -- exactly conv(fd_group_norm(x)), without the normalised tensor.  Replaces the GroupNorm + SiLU
   * in front of every ResnetBlock2D conv (diffusers; UNet and VAE). */
  const void* gi_affine;
  int gi_silu;
  /* Two-level batch (the 4-wave kernel, batch > 1): z -> (zo, zi) = (z / batch_inner, z % batch_inner); A, B and C
   * sit at zi * strideX + zo * strideX_o.  batch_inner <= 1: one level (z * strideX).  batch_inner > 1 takes no
   * residual, row bias, LayerNorm partials or GroupNorm statistics (FD_ERR_SHAPE). */
  int batch_inner;
  long long strideA_o, strideB_o, strideC_o;
  /* Per-row-group B operand (cross-attention as two GEMMs: each image row of a batched forward multiplies its own
   * prompt's matrices).  bsel_rows > 0: rows [g * bsel_rows, (g + 1) * bsel_rows) use slot
   * s = bsel_mod > 0 ? g % bsel_mod : g, i.e. B + s * bsel_strideB and ln_c / bias + s * bsel_strideN
   * (bsel_strideN 0: shared).  bsel_rows % 256 == 0 (no tile straddles two groups), batch 1. */
  int bsel_rows, bsel_mod;
  long long bsel_strideB, bsel_strideN;
  /* act == FD_ACT_SOFTMAX (attention probabilities straight from the score GEMM): the N columns are groups of
   * sm_group = 80 (one head's keys, two heads per 160-column tile); in each group the first sm_len (<= 80) columns
   * become softmax over those values of the epilogue before the activation (LayerNorm fold, bias, alpha), the rest
   * are written as 0.  N % 160 == 0, no residual / row bias / GEGLU, 16-bit output. */
  int sm_group, sm_len;
  /* up_phase = 1: a nearest x2 upsample conv (upsample = 1, Hout = 2 Hin, Wout = 2 Win) with its weights in the
   * four-phase form of pack_conv3x3_up2 ([4 * Cout][4 * Cin], B = those, ldb >= 4 Cin, K = 4 Cin): output pixel
   * (2i + a, 2j + b) = sum over the 2 x 2 source pixels (i + a - 1 + {0, 1}, j + b - 1 + {0, 1}) -- 16 taps per
   * 2 x 2 output pixels instead of 36, the same function up to the rounding of the summed weights.  Only the
   * halo-staged kernel runs it (FD_ERR_SHAPE when it cannot: Win < 16, Hin < 8, Cout not a multiple of 128 / 160);
   * no concat source, no gi_affine; gn_part blocks are (image, phase, 256- or 128-pixel tile). */
  int up_phase;
  /* Extents fd_gemm checks on the host before any launch (FD_ERR_SHAPE when short, also for 0 with the pointer set):
   * rowbias_rows = row groups the rowbias table holds, >= ceil(M / rows_per_group); residual_rows = rows of ldr
   * elements readable from residual, >= M + (batch - 1) * ceil(strideR / ldr).  A ragged tile's rows past the last
   * image are masked in every epilogue; these make an undersized table a returned error instead of a silent
   * over-read (the r04 halo-conv row-bias fault, profiles/r04zc_serialized_fault.log). */
  long long rowbias_rows, residual_rows;
} fd_gemm_params;

int fd_gemm(fd_gemm_params* p, void* stream);  /* writes only p->gn_done */
/* 3x3 stride-1 pad-1 convs (Cin % 64 == 0, Cout % 128 or 160 == 0, no concat source) run on the halo-staged kernel
 * (csrc/conv_halo.hip: each input patch staged once per 64-channel chunk, 9 taps read from LDS) when it has enough
 * tiles; the choice reads m_ref, never the batched M.  Returns the rows per GroupNorm-statistics block it writes
 * (256 or 128), 0 when fd_gemm would use the implicit GEMM for this conv. */
int fd_conv_halo_plan(const fd_gemm_params* p);
/* Workgroups of the halo kernel's persistent form for this conv (one per CU, each walking a strided list of 256-row
 * tiles with the next tile's DMA under the current tile's epilogue; bitwise equal to the one-tile-per-workgroup
 * form), 0 when the conv runs one workgroup per tile or not on the halo kernel.  Knob FD_CONV_HALO_PT. */
int fd_conv_halo_pt(const fd_gemm_params* p);
/* Workspace fd_gemm needs for this launch (0 = none). */
long long fd_gemm_ws_bytes(const fd_gemm_params* p);

/* Direct convolution for the few convs with Cin < 64 (k*k*Cin in {36, 27, 8, 4}) (UNet conv_in 4->320, VAE conv_in 3->128,
 * decoder conv_in 4->512, quant_conv / post_quant_conv 1x1).  x NHWC (dtype), w fp32
 * [Cout][kh][kw][Cin], bias fp32, y NHWC (out_dtype).  in_scale multiplies x on load.
 * Replaces: cuDNN conv2d of those layers (ext:571; diffusers Encoder/Decoder conv_in). */
int fd_conv2d_direct(const void* x, const float* w, const float* bias, void* y, int nimg, int Hin, int Win,
                     int Cin, int Cout, int ksize, int stride, int pad, float in_scale, int dtype, int out_dtype,
                     void* stream);

/* 3x3 conv, stride 1, pad 1, with few output channels (Cout <= 4, Cin in {32, 64, 128}): the VAE
 * decoder's conv_out (128 -> 3).  x NHWC (dtype bf16 / f16), w fp32
 * [Cout][3][3][Cin] (tap-major like the GEMM's
 * packed conv weights), bias fp32, y NHWC [.., Cout] (out_dtype).  fp32 accumulation, direct (no im2col).
 * Replaces: cuDNN conv2d of decoder.conv_out (diffusers Decoder; pipeline_FaithDiff_tlc.py:1438). */
int fd_conv3x3_narrow(const void* x, const float* w, const float* bias, void* y, int nimg, int H, int W, int Cin,
                      int Cout, int dtype, int out_dtype, void* stream);
/* The same conv of GroupNorm(+SiLU)(x): gi_affine fp32 (scale, shift) per (image, channel) [nimg][Cin][2] from
 * fd_group_norm_affine (16-B aligned), applied to every staged input element exactly as fd_group_norm would store it
 * (zero padding after the transform) -- the decoder's conv_norm_out + SiLU + conv_out without the normalised
 * tensor.  Replaces: GroupNorm, SiLU and conv_out of the diffusers Decoder (pipeline_FaithDiff_tlc.py:1438). */
int fd_conv3x3_narrow_gn(const void* x, const float* w, const float* bias, const float* gi_affine, int gi_silu,
                         void* y, int nimg, int H, int W, int Cin, int Cout, int dtype, int out_dtype, void* stream);

/* ---------------------------------------------------------------------------------------------
 * GroupNorm over NHWC x[nimg][HW][C] (32 groups typical), fp32 statistics, optional fused SiLU.
 * Two launches (partial stats, then normalise); `ws` must hold fd_group_norm_ws_bytes() bytes.
 * Replaces: torch native_group_norm (+ silu) in ResnetBlock2D.norm1/2, Transformer2DModel.norm,
 *   conv_norm_out, ControlNetConditioningEmbedding.norm_in (ext:208,215), VAE attention group_norm.
 * ------------------------------------------------------------------------------------------- */
long long fd_group_norm_ws_bytes(int nimg, int HW, int C, int groups);
int fd_group_norm(const void* x, void* y, const float* gamma, const float* beta, int nimg, int HW, int C,
                  int groups, float eps, int silu, int dtype, void* ws, void* stream);
/* fd_group_norm when the producing fd_gemm wrote the statistics (fd_gemm_params.gn_part, gn_done = part_rows):
 * part [nimg][HW / part_rows][groups] float2 (sum, sumsq), part_rows 256 or 128 (or the chunk rows of
 * fd_concat_channels_gn: any power of two); stats: nimg * groups float2 of caller
 * memory, written.  HW % part_rows == 0.  Saves the statistics pass over x (one full read).  Same arithmetic as
 * fd_group_norm except the summation order of the statistics (identical to it with fd_concat_channels_gn's
 * partials). */
int fd_group_norm_partials(const void* x, void* y, const float* gamma, const float* beta, int nimg, int HW, int C,
                           int groups, float eps, int silu, const void* part, int part_rows, void* stats, int dtype,
                           void* stream);
/* GroupNorm as a per-(image, channel) affine for a consumer that applies it itself (fd_gemm_params.gi_affine):
 * statistics from the producer's partials (part != NULL, part_rows = gn_done) or from x (a gn_partial pass; ws of
 * fd_group_norm_ws_bytes), then affine[i][c] = (rstd * gamma[c], beta[c] - mean * rstd * gamma[c]) -- the exact
 * scale / shift fd_group_norm applies.  affine: fp32 [nimg * C + 64][2]. */
int fd_group_norm_affine(const void* x, const void* part, int part_rows, const float* gamma, const float* beta,
                         int nimg, int HW, int C, int groups, float eps, void* ws, void* affine, int dtype,
                         void* stream);

/* LayerNorm fused with the per-row e4m3 quantization of fd_quant_rows_e4m3 (use_fp8 model): the row is
 * normalised, rounded to dtype, then q[m][:] = e4m3_RNE(y * 448 / amax_m), scale[m] = amax_m / 448 -- bitwise
 * equal to fd_layer_norm followed by fd_quant_rows_e4m3, without the 16-bit round trip.  ldq % 8 == 0.
 * Replaces: norm1/2/3 of BasicTransformerBlock (diffusers) ahead of the quantized UNet's Linears. */
int fd_layer_norm_e4m3(const void* x, long long ldx, void* q, long long ldq, float* scale, const float* gamma,
                       const float* beta, int M, int C, float eps, int dtype, void* stream);

/* ---------------------------------------------------------------------------------------------
 * fp8 (OCP e4m3) GEMM on the block-scaled MFMA v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales):
 *   C[m][n] = out( act(a_scale[m] * w_scale * sum_k A8[m][k] * W8[n][k] + bias[n]) + residual[m][n] )
 * act: FD_ACT_* as fd_gemm (GEGLU: W rows packed [16 hidden | 16 gate] per 32, N % 32 == 0, N/2 output columns).
 * A8 [M][lda] e4m3 activations with per-row fp32 scales from fd_quant_rows_e4m3; W8 [N][ldw] e4m3 weights
 * (the reference's unscaled quantize_8bit bytes, utils/system.py:13-32, w_scale = 1).  Out dtype bf16 / f16 /
 * f32 (residual, if given, in the out dtype; not with f32).  Requires K % 16 == 0, lda % 16 == 0, ldw % 16 == 0.
 * Replaces: the fp16 autocast matmul on upcast float8_e4m3fn weights behind every nn.Linear of the
 *   quantized UNet (pipeline_FaithDiff_tlc.py:1349 autocast, utils/system.py:20 .to(float8_e4m3fn)). */
int fd_gemm_e4m3(const void* A8, long long lda, const float* a_scale, const void* W8, long long ldw, float w_scale,
                 void* C, long long ldc, int M, int N, int K, const float* bias, const void* residual, long long ldr,
                 int act, int out_dtype, void* stream);

/* ---------------------------------------------------------------------------------------------
 * MX-fp8 (OCP MX e4m3: one E8M0 scale byte per 32 consecutive K elements of a row) -- the use_fp8 model's
 * activation format when the producers write it directly (flash attention, GEGLU, LayerNorm; no separate
 * quantization launch).  Scale rule (every producer): E = least exponent with amax_block <= 448 * 2^E,
 * q = RNE_e4m3(v * 2^-E), byte = E + 127 (all-zero block: 127).
 *
 * GEMM: C = out( act(w_scale * sum_k (A8[m][k] * 2^(as[m][k/32] - 127)) * W8[n][k] + bias[n]) + residual[m][n] ),
 * on v_mfma_scale_f32_16x16x128_f8f6f4 with the A block scales as the MFMA's per-lane scale operand.  A8 [M][lda]
 * e4m3, as [M][ldas] bytes (ldas % 4 == 0, >= K / 32, 4-B aligned); W8 as fd_gemm_e4m3.  out_dtype FD_BF16 / FD_F32,
 * or FD_MXE4M3: C gets e4m3 bytes [M][ldc] of the (GEGLU) output and c_bs [M][ldcs] its block scales (no residual;
 * M % 256 == 0 and N_out % 64 == 0).  Requires K % 128 == 0.  Replaces: as fd_gemm_e4m3. */
enum { FD_MXE4M3 = 3 };
int fd_gemm_mxe4m3(const void* A8, long long lda, const void* a_bs, long long ldas, const void* W8, long long ldw,
                   float w_scale, void* C, long long ldc, void* c_bs, long long ldcs, int M, int N, int K,
                   const float* bias, const void* residual, long long ldr, int act, int out_dtype, void* stream);
/* x[M][K] (bf16 / f16 / f32, row stride ldx) -> MX e4m3 q [M][ldq] + scales s [M][lds].  K % 32 == 0. */
int fd_quant_rows_mx(const void* x, long long ldx, void* q, long long ldq, void* s, long long lds, int M, int K,
                     int dtype, void* stream);
/* LayerNorm (as fd_layer_norm, output rounded to bf16) written as MX e4m3 -- bitwise fd_layer_norm then
 * fd_quant_rows_mx.  C % 32 == 0; dtype FD_BF16 only. */
int fd_layer_norm_mx(const void* x, long long ldx, void* q, long long ldq, void* s, long long lds, const float* gamma,
                     const float* beta, int M, int C, float eps, int dtype, void* stream);

/* Per-row e4m3 quantization of x[M][K] (row stride ldx, bf16 / f16): scale[m] = amax_m / 448,
 * q[m][k] = e4m3_RNE(x[m][k] * 448 / amax_m) into q (row stride ldq bytes).  Requires K % 16 == 0,
 * ldx % 8 == 0, ldq % 16 == 0.  Activation side of fd_gemm_e4m3 (the reference has no counterpart: it
 * computes on fp16 activations; the tolerance of this leg is stated separately). */
int fd_quant_rows_e4m3(const void* x, long long ldx, void* q, long long ldq, float* scale, int M, int K, int dtype,
                       void* stream);

/* LayerNorm over the last dim of x[M][C] (row stride ldx), fp32 stats; y[M][C] (ldy).
 * Replaces: torch layer_norm in BasicTransformerBlock.norm1/2/3 and ResidualAttentionBlock.ln_1/2
 *   (ext:243,248,258-259). */
int fd_layer_norm(const void* x, long long ldx, void* y, long long ldy, const float* gamma, const float* beta,
                  int M, int C, float eps, int dtype, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Flash attention forward, head_dim 64, online softmax in fp32, MFMA for QK^T and PV.
 * q/k/v/o are row-major token matrices; head h of batch b lives at
 *   q + b*q_bstride + t*ldq + h*64 (same for o); k/v use batch index (kv_mod ? b % kv_mod : b), so
 *   the cross-attention K/V of the [neg, pos] prompt pair serve every tile of a batched forward.
 *   Lk may be any size (masked tail).  causal != 0: query i sees keys <= i (CLIP text encoders).
 * Replaces: SDPA (flash / mem-efficient) behind diffusers AttnProcessor2_0 for attn1 (self,
 *   T = 4096 / 1024 per tile) and attn2 (cross, Lk = 77) of all 70 BasicTransformerBlocks.
 * ------------------------------------------------------------------------------------------- */
int fd_flash_attn(const void* q, long long ldq, long long q_bstride, const void* k, long long ldk,
                  long long k_bstride, const void* v, long long ldv, long long v_bstride, void* o, long long ldo,
                  long long o_bstride, int batch, int heads, int Lq, int Lk, int kv_mod, int causal, float scale,
                  int dtype, void* stream);
/* fd_flash_attn (d = 64, bf16 in) with the output written as MX e4m3 for the use_fp8 model's out-projection
 * (fd_gemm_mxe4m3): o8 e4m3 bytes at o8 + b * obs + q * ldo + h * 64 (ldo, obs in bytes, % 4 == 0), E8M0 scales of
 * the (query, head)'s two 32-column blocks at osb[b * osbs + q * ldos + 2 h + {0, 1}], quantized from the fp32
 * normalised output (fd_quant_rows_mx's rule). */
int fd_flash_attn_mx(const void* q, long long ldq, long long q_bstride, const void* k, long long ldk,
                     long long k_bstride, const void* v, long long ldv, long long v_bstride, void* o8, long long ldo,
                     long long o_bstride, void* osb, long long ldos, long long os_bstride, int batch, int heads, int Lq,
                     int Lk, int kv_mod, int causal, float scale, int dtype, void* stream);

/* The information transformer's nn.MultiheadAttention(640, 8) with batch_first=False fed
 * (L=B, N=HW, E) (ext:242,251-254,576-577): for each pixel n, softmax attention over the L rows of
 * each of `groups` consecutive row groups (one group = one tile's CFG pair when tiles are batched).
 * qkv: [groups*L][N][3E] (in_proj output), o: [groups*L][N][E].  L <= 2 (the CFG pair), head dim 80
 * (FaithDiff's 640 / 8); exact for distinct rows. */
int fd_mha_seq_axis(const void* qkv, void* o, int L, int groups, int N, int E, int heads, int dtype, void* stream);

/* Single-head flash attention with head_dim 512 (the VAE mid-block Attention: diffusers Attention with one head
 * of 512 channels, upcast softmax -- AutoencoderKL decode, pipeline_FaithDiff_tlc.py:1436-1442, and the VAE /
 * FaithDiff denoise encoders, ext:39-196).  q/k/v: token rows of length >= 512 with row stride ld (elements; the
 * qkv projection output [L][1536] gives q, k = q + 512, v = q + 1024), batch stride bs; o: [L][ldo] rows, batch
 * stride obs.  L may be any size (masked tail).  No [L, L] buffer is formed.  16-B aligned q/k/v, ld % 8 == 0. */
int fd_flash_attn_d512(const void* q, const void* k, const void* v, long long ld, long long bs, void* o,
                       long long ldo, long long obs, int batch, int L, float scale, int dtype, void* stream);
/* The same attention on 8-wave workgroups (128 queries per K/V tile fetch, half the operand bytes per flop of
 * fd_flash_attn_d512) with the keys of each query block split over `ks` workgroups.  ks > 1: each split writes
 * its O / l (fp32) and log2-sum-exp into `part` (>= batch * ks * L * 513 floats, 16-B aligned) and a second launch
 * merges the splits in split order into o (then o, ldo and obs must be 16-B / 8-element aligned).  ks = 1 writes o
 * directly and `part` may be NULL.  fd_flash_attn_d512_ksplit returns the split count the library plans for
 * (batch, L): enough workgroups for the 256 CUs, at least 4 key tiles of 32 per split. */
int fd_flash_attn_d512_ksplit(int batch, int L);
int fd_flash_attn_d512_split(const void* q, const void* k, const void* v, long long ld, long long bs, void* o,
                             long long ldo, long long obs, int batch, int L, float scale, int dtype, float* part,
                             long long part_floats, int ks, void* stream);

/* Row softmax of fp32 scores s[R][C] (scaled by `scale`) into p[R][ldp] (dtype).  With fd_gemm this forms
 * a materialised single-head attention (kept for head dims other than 512; the VAE uses fd_flash_attn_d512). */
int fd_softmax_rows(const float* s, void* p, int R, int C, long long ldp, float scale, int dtype, void* stream);

/* Cross-attention as two GEMMs (attn2 of every BasicTransformerBlock, diffusers Attention called from
 * unet_2d_condition_vae_extension.py:571-690 through pipeline_FaithDiff_tlc.py:1350-1360; the prompt K / V are
 * fixed for the whole denoise loop).  Per prompt row r the score matrix B1[r] = scale * K_r,h . W_q' (row
 * (r * heads + h) * slot + j per head h and key j, written by a batched fd_gemm) gets its LayerNorm-fold
 * constants here: c[n] = sum_k B1[n][k] (stored values, fixed order), d[n] = scale * K_r[j][h*64..] . dq[h*64..]
 * (dq = W_q . beta fp32; 0 for pad keys j >= Lk).  kv: K rows of prompt r at kv + r * kv_rstride + j * ldkv
 * (head h at column h * 64).  rows = R * heads * slot.  dtype: of B1 and kv. */
int fd_xattn_consts(const void* B1, long long ldb, int rows, int K, const void* kv, long long ldkv,
                    long long kv_rstride, const float* dq, int heads, int slot, int Lk, float scale, float* c,
                    float* d, int dtype, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Elementwise / layout helpers (all HBM-bound).
 * ------------------------------------------------------------------------------------------- */
/* y[m][0:C1] = a[m][0:C1], y[m][C1:C1+C2] = b[m][0:C2]  (up-block skip concat, diffusers
 * CrossAttnUpBlock2D / UpBlock2D torch.cat) */
int fd_concat_channels(const void* a, int C1, const void* b, int C2, void* y, long long M, int dtype, void* stream);
/* fd_concat_channels over M = nimg * HW rows plus the GroupNorm statistics of y for its consumer (the up-block
 * resnet's norm1): part[(i * HW / R + k) * groups + g] = (sum, sum of squares) of image i, R-row chunk k, group g,
 * R = fd_group_norm_chunk_rows(nimg, HW) -- fd_group_norm's own statistics pass, bit for bit, fused into the copy.
 * part: nimg * (HW / R) * groups float2.  Consumer: fd_group_norm_partials / fd_group_norm_affine with
 * part_rows = R.  Replaces: torch.cat + the first half of native_group_norm (diffusers UpBlock2D resnets). */
int fd_group_norm_chunk_rows(int nimg, int HW);
int fd_concat_channels_gn(const void* a, int C1, const void* b, int C2, void* y, int nimg, int HW, int groups,
                          void* part, int dtype, void* stream);
/* y = act(x) elementwise, n elements; also casts dtype -> out_dtype (act 0 = copy/cast). */
int fd_unary(const void* x, void* y, long long n, int act, int dtype, int out_dtype, void* stream);
/* y[m][n] = x[m][n] (+ a[m][n] if a != NULL), general row strides; dtype cast allowed. */
int fd_add_strided(const void* x, long long ldx, const void* a, long long lda, void* y, long long ldy, int M, int N,
                   int dtype, int out_dtype, void* stream);
/* y[m][n] = alpha * x[m][n] + beta * z[m][n] (bf16/f16, N % 8 == 0, 16-B aligned rows; y may alias z).
 * Replaces the RRDB residual `out * 0.2 + x` of the BSRNet pre-pass (bsrnet_arch.py:72-76). */
int fd_axpby(const void* x, long long ldx, const void* z, long long ldz, void* y, long long ldy, int M, int N,
             float alpha, float beta, int dtype, void* stream);
/* NCHW <-> NHWC transposes (dtype in, out_dtype out; scale applied). */
int fd_nchw_to_nhwc(const void* x, void* y, int nimg, int C, int HW, float scale, int dtype, int out_dtype,
                    void* stream);
int fd_nhwc_to_nchw(const void* x, void* y, int nimg, int C, int HW, float scale, int dtype, int out_dtype,
                    void* stream);
/* 2-D transpose y[C][R] = x[R][C] with batch (VAE attention V^T). */
int fd_transpose(const void* x, long long ldx, void* y, long long ldy, int R, int C, int batch, long long sx,
                 long long sy, int dtype, void* stream);

/* SDXL time / micro-conditioning features (diffusers get_timestep_embedding, flip_sin_to_cos, shift 0;
 * ext:543-561): tfeat[b][0:320] = sinusoid(t[b]); afeat[b] = [text_embeds[b] (1280) |
 * sinusoid_256(time_ids[b][0..5])].  t, time_ids, text_embeds fp32 on device; outputs dtype. */
int fd_time_features(const float* t, const float* time_ids, const float* text_embeds, void* tfeat, void* afeat,
                     int batch, int dtype, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Denoise-loop fusions (pipeline_FaithDiff_tlc.py:1271-1409).  The latent canvas is fp32 NCHW
 * [4][H][W]; tile t of the TLC grid has origin (row_org[t / nc], col_org[t % nc]) -- the row-major
 * Cartesian order LocalAttention.grids (:160-205) produces; tiles [tile_begin, tile_begin+ntiles)
 * are this call's (a rank's shard when tiles are spread over GPUs).
 * ------------------------------------------------------------------------------------------- */
/* grids + CFG duplicate + EulerDiscreteScheduler.scale_model_input (:1326,1334-1336):
 * out NHWC dtype [ntiles*cfg][kh*kw][4] = canvas tile / scale, correctly rounded fp32 division, where the
 * argument `sigma` carries scale = (sigma^2 + 1)^0.5 as torch computes it in fp32 from the sigma (ops.py
 * euler_scale_divisor); must be > 0. */
int fd_tlc_scale_input(const float* canvas, const int* row_org, int nr, const int* col_org, int nc, int H, int W,
                       int kh, int kw, int tile_begin, int ntiles, int cfg, float sigma, void* out, int dtype,
                       void* stream);
/* The same, also writing the step's UNet timestep into t_out[0 .. t_n) (any t_n >= 0; the `t` row of the UNet call,
 * :1350-1360) from inside the same launch: the denoise loop's per-step host-side fill of the timestep buffer (a
 * separate elementwise launch) is gone. */
int fd_tlc_scale_input_t(const float* canvas, const int* row_org, int nr, const int* col_org, int nc, int H, int W,
                         int kh, int kw, int tile_begin, int ntiles, int cfg, float sigma, void* out, int dtype,
                         float* t_out, int t_n, float timestep, void* stream);
/* CFG combine (+ rescale_noise_cfg when guidance_rescale > 0, :286-305,1363-1369) and the Euler step
 * (:1373; gamma = 0, fp32): eps NHWC [ntiles*cfg][kh*kw][4] (uncond row first), x = canvas tile,
 * out_tiles fp32 NCHW [ntiles][4][kh][kw] = x + ((x - (x - sigma*e)) / sigma) * (sigma_next - sigma). */
int fd_tlc_cfg_euler_step(const void* eps, const float* canvas, const int* row_org, int nr, const int* col_org, int nc,
                          int H, int W, int kh, int kw, int tile_begin, int ntiles, int cfg, float guidance,
                          float guidance_rescale, float sigma, float sigma_next, float* out_tiles, int dtype,
                          void* stream);
/* LocalAttention.grids_inverse (:230-252): canvas[c][y][x] = sum_t tile*w / sum_t w over the covering
 * tiles in tile order, each product in fp64 rounded to fp32 per add exactly like the reference's
 * fp32 canvas += tile * fp64 weight.  weights fp64 [kh][kw] (_gaussian_weights, :207-228). */
int fd_tlc_blend(const float* tiles, const double* weights, const int* row_org, int nr, const int* col_org, int nc,
                 int C, int H, int W, int kh, int kw, float* canvas, void* stream);
/* LocalAttention.grids on the NHWC image-latent canvas [H][W][C] (:1257) + CFG duplicate (:1335):
 * out [ntiles*cfg][kh][kw][C]. */
int fd_tlc_grids_nhwc(const void* canvas, const int* row_org, int nr, const int* col_org, int nc, int H, int W, int C,
                      int kh, int kw, int tile_begin, int ntiles, int cfg, void* out, int dtype, void* stream);
/* prepare_latents + start_point 'lr' (:820-835, 1271-1276): moments NHWC [HW][8] (VAE quant_conv
 * output), post_eps/noise fp32 NCHW [4][HW];  out = a * (mean + exp(0.5 clamp(logvar,-30,20)) *
 * post_eps) * scaling + b * noise * init_sigma   (a, b = DDPM add_noise coefficients at t = 999);
 * start_lr == 0: out = noise * init_sigma. */
int fd_vae_sample_add_noise(const void* moments, const float* post_eps, const float* noise, float* out, int HW,
                            float scaling, float init_sigma, float a, float b, int start_lr, int dtype, void* stream);
/* VaeImageProcessor.postprocess (:1451): uint8 = round(clamp(x/2 + 0.5, 0, 1) * 255). */
int fd_postprocess_u8(const void* x, void* y, long long n, int dtype, void* stream);

/* Tiled VAE / denoise-encoder seam blend (diffusers AutoencoderKL.blend_v/blend_h; FaithDiff
 * Encoder.blend_v/blend_h, ext:150-162), in place on NHWC tile b from neighbour a (vertical: a above
 * b; horizontal: a left of b); e = min(extent, overlapping dims). */
int fd_blend_edge(const void* a, void* b, int Ha, int Wa, int Hb, int Wb, int C, int extent, int vertical, int dtype,
                  void* stream);

/* CLIP text embeddings (transformers CLIPTextEmbeddings behind encode_prompt, pipeline:587-598):
 * out[b*L + l][:] = tok[ids[b*L + l]][:] + pos[l][:]; ids int32 on device, tables [vocab][D] / [L][D] in dtype. */
int fd_embed_tokens(const int* ids, const void* tok, const void* pos, void* out, int batch, int L, int D, int vocab,
                    int dtype, void* stream);

/* Launch-planner knobs (csrc/knobs.hip): one table of tested defaults compiled into the library, which never reads
 * the environment.  Tests and measurement scripts switch an entry by name (e.g. "FD_GEMM256" = 0 to compare gemm8
 * with gemm256 bitwise) and restore it; the product path never calls these.  Unknown name: FD_ERR_ARG. */
int fd_set_knob(const char* name, int value, int* previous);
int fd_get_knob(const char* name, int* value, int* dflt);
const char* fd_knob_name(int id); /* NULL past the last knob */
void fd_reset_knobs(void);

/* Split-K hand-off health.  The pairwise split-K forms (gemm8 S = 2, the halo conv's channel split) hand a partial tile
 * from one workgroup to its partner through a flag with a bounded wait; a wait that times out (should never happen:
 * the publisher is already running) poisons its tile with NaN and is counted here.  After a timeout that tile's
 * counter / flag slot is stale, so the host must re-zero the first 256 KiB of every split-K workspace
 * (fdhip/ops.py split_k_health does, and raises).  Synchronous; *timeouts = count since the last reset.
 * fd_splitk_test_drop(1) is a test hook only: every publisher skips its flag (forces the timeout path). */
int fd_splitk_health(unsigned* timeouts, int reset);
int fd_splitk_test_drop(int drop);

/* library / device checks */
int fd_device_check(void);
const char* fd_version(void);

#ifdef __cplusplus
}
#endif
#endif
