// Kernel-argument structs shared between translation units (device-side views of the public
// descriptors in include/dfcsa.h).
#pragma once
#include "common.h"
#include "dfcsa.h"

struct ConvSeg {
  const void* ptr;
  int dh, dw;
};

// BatchNorm finalisation folded into a conv epilogue (dfcsa_conv_gemm_bn): the launch's statistics
// rows are reduced by its own last workgroups (two ticket levels) and finalised as dfcsa_bn_finalize
// (training) does.  on == 0: no fold.
struct BnFold {
  int on, C, GS, ng, ncb, cw;   // channels finalised, rows per group, groups, column blocks, block width
  unsigned* cnt;                // ncb * ng level-1 tickets, then ncb level-2 tickets (zero, re-zeroed)
  double* scr;                  // [ncb][ng][2][cw] group sums (write-through hand-off)
  int count;
  const float* bias;
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  int64_t* nbt;
  float momentum, eps;
  float* scale;
  float* shift;
  float* mean;
  float* invstd;
};

struct ConvGemmArgs {
  int M, N, K, Kpad, Cseg, nseg;
  ConvSeg seg[DFCSA_MAX_SEG];
  int Ho, Wo, Hi, Wi, stride;
  DivMod dm_hw, dm_w, dm_cseg;
  const void* Bw;
  const float* bias;
  int mode, ndest;
  void* dest[3];
  int Nd, accumulate;
  float* stats;
  int Hout, Wout;
  int dbg;   // timing experiments only (knob 15): 1 = A operand from the zero page, 2 = B
  // split-K (dfcsa_conv_desc.work): fp32 partial tiles of ksplit K ranges of kper 64-deep stages,
  // summed in split order by the epilogue launch; kwork == nullptr: never split
  float* kwork;
  int64_t kwork_floats;
  int ksplit, kper;
  unsigned* kcnt;   // stream-K ping-pong launch: one ticket per output tile (zero, re-zeroed)
  BnFold fold;
};

struct WgradArgs {
  int M, NI, NJ, Cg, ng;
  const void* g_ptr[3];
  int Cseg, nseg;
  ConvSeg seg[DFCSA_MAX_SEG];
  int Ho, Wo, Hi, Wi, stride;
  DivMod dm_hw, dm_w, dm_cseg, dm_cg;
  float* slab;
  int mchunk;
  // fused split-K reduction (fuse = 1): destination mapping of dfcsa_wgrad_reduce, split count,
  // ticket counters of this launch's output tiles (zero on entry, re-zeroed by each tile's last
  // arriving workgroup)
  int fuse, nsplit, layout, ntaps, Ctot, Creal, ndst;
  float* dst[3];
  unsigned* cnt;
  // simple geometry (stride 1, input grid = output grid, shifts in [-1, 1]): the LDS-DMA kernel
  // tracks each X slot's (row, column) incrementally, 64 pixels per stage = adv_w columns and
  // adv_h rows (mod H)
  int simple, adv_w, adv_h;
  // cooperative split-K reduction (coop = 1, the whole grid co-resident): every split publishes its
  // partial tile, waits at the tile's ticket for the others, then reduces ONE slice of the tile over
  // all splits in split order and adds it into dst (no slab reduction launch)
  int coop;
  // layout 2: bias gradients (column sums of G) added by the small fp32 kernel, bdst[0] != NULL
  float* bdst[3];
};

// profiling hook (prof.cpp)
struct ProfScope {
  int cls;
  hipStream_t st;
  double flops;
  bool on;
  ProfScope(int cls, hipStream_t st, double flops);
  ~ProfScope();
};

extern int g_wgrad_target;
extern int g_wgrad_waves;
extern int g_wgrad_noglds;
extern int g_wgrad_narrow;
extern int g_wgrad_fuse_all;
extern int g_wgrad_fuse_max;
extern int g_wgrad_nst;
extern int g_wgrad_noglds_f32small;
extern int g_wgrad_big;
extern int g_wgrad_wide_small;
extern int g_wgrad_halo;
extern int g_wgrad_reduce_old;
extern int g_wgrad_nst64;
extern int g_wgrad_bd;
extern int g_wgrad_bd_nst;
extern int g_wgrad_coop_launches;
extern int g_wgrad_coop;   // knob 31: cooperative in-launch split-K reduction (0 = separate reduction launch)
extern int g_small8;
extern int g_lsa_rows_old;  // knob 28: 1 = the item-owner LightSelfAttention upsample-backward row kernel
extern int g_lsa_pool_direct;  // knob 47: one wave per window for P >= 16 (dfcsa_lsa_pool_direct, default 1)
extern int g_lsa_key_centre;
extern int g_lsa_cols_flash;
extern int g_gn_chunk;   // knob 50: 128-channel chunks in the fused GroupNorm reductions (default 1)   // knob 49: fused column pass + prep for the bf16 flash layers (default 1)  // knob 48: mean-key centred dQ in the bf16 pooled-attention backward (default 1)
extern int g_lsa_pool_one_slice;  // knob 46: small pool windows in one row slice (default 1)
extern int g_lsa_cols_nt;  // knob 35: 256 = the 256-thread LightSelfAttention upsample-backward column kernel
extern int g_wgrad_nosimple;
// n ticket counters for a last-arriver hand-off (ring in block_ew.hip; nullptr on failure)
unsigned* dfcsa_ticket_alloc(int n);
// n doubles of last-arriver hand-off scratch (ring in block_ew.hip; nullptr on failure)
double* dfcsa_scratch_alloc(int64_t n);
extern int g_fra_generic;
extern int g_fra_occ;
extern int g_ew_tile_elems;

// DFCSA_SHAPELOG=1: one stderr line per conv / wgrad launch (shape analysis against a kernel
// trace, tools/shape_trace.py); off by default
bool dfcsa_shapelog();

// bf16 pooled-attention backward pieces shared by fra.hip and lsa.hip (dfcsa_lsa_flash_bwd_up): the
// work pointers plus the one / key-sum launch, and the MFMA kernels after the prep step
int lsa_flash_prepare_ext(int B, int N, int C, int Cq, int ldq, const void* qkv, void* work, int64_t work_bytes,
                          bf16_t** dO16, float** r, int* nch, const float** kb, hipStream_t st);
void lsa_flash_bwd_core(int B, int N, int C, int Cq, int ldq, const void* qkv, const float* lse, void* dqkv, void* work,
                        const float* kb, hipStream_t st);
