// One-wave-per-SIMD MFMA GEMM for gfx950 — the frozen-base GEMMs of the QLoRA step:
//
//   forward   y  = x·Wᵀ (+ residual)      A = x [M, K],  B = W  [N, K]   (NT)
//   backward  dX = dY·W (+ C)             A = dY [M, K], B = W  [K, N]   (BT: W used as stored)
//
// W is bf16, or (W4) the NF4 4-bit codes of a QLoRA base: the K9 "NF4 dequant-GEMM" — the codes are
// expanded to bf16 inside the kernel, between the global load and the LDS B image, so no bf16 copy of
// the frozen base ever exists in HBM (reference: BitsAndBytesConfig(load_in_4bit, nf4, double quant),
// Fine-Tuning/qwen3-8b-qlora-dist.py:102-110).
//
// Design (profiles/gemm4w_*.txt, profiles/r3/, profiles/r4/):
//  * 256 threads = 4 waves as 2 (M) × 2 (N), one wave per SIMD; a wave owns a BM/2 × BN/2 output block
//    of v_mfma_f32_16x16x32_bf16 accumulators (up to 256 fp32 per lane) held in AGPRs.  The MFMAs
//    are one-instruction asm statements with the accumulator a tied "+a" operand (with the builtin,
//    hipcc split the accumulator phis between the two K-halves and shuffled ~48 v_accvgpr_mov/read/
//    write per K-tile through the MFMA results).  A fragment register is rewritten ≥ 16 MFMAs after
//    its last reader; one wave per SIMD, so no partner's MFMAs sit between; the epilogue's AGPR reads
//    sit behind 16 wait states.
//  * BN = 256 / 192 / 128 and BM = 256 / 128 chosen per shape by one cost model (gemm4w_cfg).
//  * A (and bf16 B): global → LDS only by LDS-DMA (buffer_load … lds, 1 KB per wave-instruction,
//    whole 128-B lines), STAGES K-tile stages (2 at 256 × 256: 128 KB; 3 where they fit 160 KB).
//    Per K-tile one compile-time-unrolled stream of KT MFMAs (first K-half on fA, second on fB):
//      - the first R MFMAs each carry one fragment read of this tile's second half (into fB);
//      - barrier 1 (lgkmcnt(0)): nobody reads stage t % STAGES any more → its refill with tile
//        t + STAGES is spread over the middle MFMAs;
//      - barrier 2 (vmcnt): tile t + 1 has landed;
//      - the last R MFMAs each carry one fragment read of tile t + 1's first half (into fA).
//    The first half walks (i, j) in shells of max(i, j), so MFMA k waits only on reads issued ≥ 14
//    MFMAs earlier.
//  * W4 B operand (the NF4 base): per K-tile every lane expands ONE 64-element quant block (32 in the
//    128-wide tiles).  Its 4-bit codes and fp32 absmax are LDS-DMA'd into a 2-slot ring one K-tile
//    ahead (counted by the same explicit vmcnt waits as the A DMAs; each lane reads back its own
//    bytes); the lane builds the block's scaled 16-entry table T[i] = bf16(code_i · absmax) —
//    bit-identical to the bitsandbytes / nf4_dequant expansion — as lo-byte and hi-byte planes
//    (4 + 4 dwords), expands its codes with v_perm_b32 byte lookups (3 VALU per element) and ds_writes
//    the bf16 chunks into the SAME LDS B image the bf16 path DMAs.  At BM = 256 a lane expands 0.5
//    elements per MFMA it issues: ≈1.8 VALU per 16x16x32 MFMA, cut into ≤2-VALU micro-ops placed one
//    per MFMA.  The B bytes fetched drop 4× and the B LDS-DMAs disappear.  Codes are stored pre-tiled
//    ("g4w" layout, NF4Weight.g4w_pack): [N/64][K/64][2][64 rows][16 B], nibble b of byte j = element
//    j + 4b of an 8-element chunk.
//  * NT images: 1 KB subtiles of 8 rows × 64 k, 16-B chunk c of row r at slot 8r + (c ^ f(r)), f(r) =
//    r & 6 for the DMA'd images, r for the W4 B image (the expanding lanes write 8 rows × one chunk per
//    ds_write group: conflict-free).  Both read conflict-free by ds_read_b128.  BT image: 64 k-rows ×
//    2·BN bytes with the 32-B column pairs XOR-permuted by h(k) = (k & 3) | ((k >> 1) & 4), read as the B
//    operand by two ds_read_b64_tr_b16 per fragment.  DMA'd swizzles are applied on the source address.
//  * XCD-aware tile order: the m-tiles of one weight panel are consecutive ids and share an XCD's L2.
//  * split-K (grids still smaller than the chip): fp32 slabs + one reduce launch (+ residual).
#pragma once
#include <type_traits>

#include "common.h"
#include "lora_epi.h"

using namespace lipa;

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int BK = 64, NT = 256;

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint64_t bytes) {
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(bytes > 0xFFFFFFFFull ? 0xFFFFFFFFull : bytes));
  void* b = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(b, 0, n, 0x00020000);
}

// NT image slot of 16-B chunk c of row r8 (0..7) in a 1 KB subtile: DMA'd images (A, bf16 B) XOR by
// r8 & 6, the lane-written W4 B image by r8
template <bool FULL>
__device__ __forceinline__ int slot_of(int r8, int c) { return 8 * r8 + (c ^ (FULL ? r8 : (r8 & 6))); }

__device__ __forceinline__ bf16x8 lds_frag(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }

// BT image: 32-B column pair c of k-row k sits at pair c ^ bt_swz(k).  A ds_read_b64_tr_b16 lane group reads
// 8 k-rows {0-3, 8-11} (+ a multiple of 4) × one 32-B pair each: at BN = 256 / 128 every row starts on bank 0
// and the 8 rows take 8 distinct 32-B bank slots through a 3-bit swizzle; at BN = 192 (384-B rows, starting on
// banks 0 / 32 alternately) a 2-bit swizzle inside each aligned group of 4 pairs (12 pairs = 3 groups: no
// pair leaves its group) gives the 8 rows distinct slots — conflict-free either way.
template <int BN>
__device__ __forceinline__ int bt_swz(int k) {
  if constexpr (BN == 192) return ((k >> 1) & 1) | ((k >> 2) & 2);
  else return (k & 3) | ((k >> 1) & 4);
}

__device__ __forceinline__ void mfma_acc(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_zero(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
}

// s_waitcnt immediate for lgkmcnt(0) (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4] << 14)
constexpr int WAIT_LGKM0 = 0 | (7 << 4) | (0 << 8) | (3 << 14);

// vmcnt wait as an asm statement (the DMAs it counts are asm too, invisible to hipcc's counters)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// one wave-instruction of LDS-DMA: 64 lanes × 16 B from rs + voff + soff into LDS [dst, dst + 1 KB);
// M0 (the LDS base, compiler-reserved) is written and restored inside the statement.  dst and soff
// are SALU values (never fresh from v_readfirstlane, so no VALU→SGPR→VMEM wait states are needed)
__device__ __forceinline__ void dma_lds(const rsrc_t& rs, uint32_t dst, uint32_t voff, uint32_t soff) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(dst), "v"(voff), "s"(rs), "s"(soff)
      : "memory");
}

// s_waitcnt immediate for vmcnt(0) alone (the full drain that register loads issued near LDS-DMAs need: a counted
// vmcnt(N > 0) is never their guard — scripts/vmcnt_audit.py, tests/test_vmcnt_audit_cpu.py)
constexpr int WAIT_VM0 = 0 | (7 << 4) | (15 << 8) | (0 << 14);

// compile-time unrolled loop: f(std::integral_constant<int, k>) for k in [K, N)
template <int K, int N>
struct Unroll {
  template <typename F>
  __device__ __forceinline__ static void run(F&& f) {
    f(std::integral_constant<int, K>{});
    Unroll<K + 1, N>::run(f);
  }
};
template <int N>
struct Unroll<N, N> {
  template <typename F>
  __device__ __forceinline__ static void run(F&&) {}
};

// Per-tile schedule tables (NA a-fragments × NB b-fragments per wave and K-half): MFMA order of a
// K-half (shells of max(i, j), then the remaining rows / columns) and the fragment-read order
// (a0 b0 a1 b1 …, then the remaining a's or b's) — MFMA k waits only on reads issued well before it.
template <int NA, int NB>
struct Sched {
  int i[NA * NB], j[NA * NB];
  int rd_a[NA + NB], rd_i[NA + NB];   // read item r: a fragment? index
};
template <int NA, int NB>
constexpr Sched<NA, NB> make_sched() {
  Sched<NA, NB> o{};
  constexpr int S = NA < NB ? NA : NB;
  int k = 0;
  for (int s = 0; s < S; ++s) {
    for (int j = 0; j <= s; ++j) { o.i[k] = s; o.j[k] = j; ++k; }
    for (int i = 0; i < s; ++i) { o.i[k] = i; o.j[k] = s; ++k; }
  }
  for (int i = S; i < NA; ++i)
    for (int j = 0; j < NB; ++j) { o.i[k] = i; o.j[k] = j; ++k; }
  for (int j = S; j < NB; ++j)
    for (int i = 0; i < S; ++i) { o.i[k] = i; o.j[k] = j; ++k; }
  int r = 0;
  for (int s = 0; s < S; ++s) {
    o.rd_a[r] = 1; o.rd_i[r] = s; ++r;
    o.rd_a[r] = 0; o.rd_i[r] = s; ++r;
  }
  for (int i = S; i < NA; ++i) { o.rd_a[r] = 1; o.rd_i[r] = i; ++r; }
  for (int j = S; j < NB; ++j) { o.rd_a[r] = 0; o.rd_i[r] = j; ++r; }
  return o;
}
constexpr Sched<8, 8> kSched88 = make_sched<8, 8>();
constexpr Sched<8, 4> kSched84 = make_sched<8, 4>();
constexpr Sched<8, 6> kSched86 = make_sched<8, 6>();
constexpr Sched<4, 8> kSched48 = make_sched<4, 8>();
constexpr Sched<4, 4> kSched44 = make_sched<4, 4>();
constexpr Sched<4, 6> kSched46 = make_sched<4, 6>();
template <int NA, int NB>
__host__ __device__ constexpr const Sched<NA, NB>& sched_of();
#define G4W_SCHED(A_, B_) \
  template <>             \
  __host__ __device__ constexpr const Sched<A_, B_>& sched_of<A_, B_>() { return kSched##A_##B_; }
G4W_SCHED(8, 8)
G4W_SCHED(8, 4)
G4W_SCHED(8, 6)
G4W_SCHED(4, 8)
G4W_SCHED(4, 4)
G4W_SCHED(4, 6)
#undef G4W_SCHED

__device__ __forceinline__ float silu_f(float g) { return g / (1.f + __expf(-g)); }

// epilogue output store (LIPA_G4W_NOSTORE: experiments only — scripts/experiments/epi_probe — keeps every value
// computed but stores only under an impossible condition, to time the epilogue's store traffic).  Non-temporal
// stores for the outputs the backward reads much later (SwiGLU g | u) won 20 µs on the isolated kernel and lost
// 0.1 ms in the step (profiles/r6/gemm4w_epilogue_probe.txt): every store is plain.
#ifdef LIPA_G4W_NOSTORE
#define G4W_ST(P, V) do { if (M < 0) *(P) = (V); } while (0)
#else
#define G4W_ST(P, V) (*(P) = (V))
#endif

// Widened epilogue stores (cdna_hip_programming.md T21, for the 16×16 layout): lane row r = lane >> 4 holds
// columns 4r .. 4r+3 of each 16-column block, so a row's 16 columns are 4 lanes × 8 B and the natural store
// is one dwordx2 per block.  v_permlane16_swap exchanges rows 1 / 3 of its first operand with rows 0 / 2 of
// its second: applied to blocks (j, j+1) it leaves lane row r holding 8 CONTIGUOUS columns —
// block j + (r & 1), columns 8·(r >> 1) .. +7 (first operand = the low 4, second = the high 4) — so one
// dwordx4 per block PAIR.  The epilogue was store-issue bound (profiles/r5/gemm4w_round_fixed_cost.txt):
// half the store (and epilogue load) instructions at the same bytes.
// (written per component on whole-vector copies: the same swaps as a loop over a[e] / b[e] element references
// miscompiled under hipcc / ROCm 7.2 — one dword loaded, the later swaps fed the earlier swaps' results)
__device__ __forceinline__ void pair_swap(f32x4& a, f32x4& b) {
  const u32x4 ua = __builtin_bit_cast(u32x4, a), ub = __builtin_bit_cast(u32x4, b);
  u32x4 oa, ob;
  {
    const auto r = __builtin_amdgcn_permlane16_swap(ua[0], ub[0], false, false);
    oa[0] = r[0];
    ob[0] = r[1];
  }
  {
    const auto r = __builtin_amdgcn_permlane16_swap(ua[1], ub[1], false, false);
    oa[1] = r[0];
    ob[1] = r[1];
  }
  {
    const auto r = __builtin_amdgcn_permlane16_swap(ua[2], ub[2], false, false);
    oa[2] = r[0];
    ob[2] = r[1];
  }
  {
    const auto r = __builtin_amdgcn_permlane16_swap(ua[3], ub[3], false, false);
    oa[3] = r[0];
    ob[3] = r[1];
  }
  a = __builtin_bit_cast(f32x4, oa);
  b = __builtin_bit_cast(f32x4, ob);
}

// ------------------------------------------------------------------ NF4 (W4) B-operand expansion
// bitsandbytes NF4 code values
constexpr float kNF4c[16] = {
    -1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
    -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
    0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f, 0.33791524171829224f,
    0.44070982933044434f, 0.5626170039176941f, 0.7229568362236023f, 1.0f};

__device__ __forceinline__ uint32_t vperm(uint32_t s0_hi, uint32_t s1_lo, uint32_t sel) {
  return __builtin_amdgcn_perm(s0_hi, s1_lo, sel);
}
// (m & a) | (~m & b), one v_bfi_b32
__device__ __forceinline__ uint32_t vbfi(uint32_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}
// f32 product, never SLP-packed into v_pk_mul_f32 (packed f32 beside MFMAs is an anti-lever on CDNA4)
__device__ __forceinline__ float vmul(float a, float b) {
  float r;
  asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {   // v_cvt_pk_bf16_f32 (RNE): a → low half
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
}

// one wave-instruction of dword LDS-DMA: 64 lanes × 4 B into LDS [dst, dst + 256 B)
__device__ __forceinline__ void dma_lds4(const rsrc_t& rs, uint32_t dst, uint32_t voff, uint32_t soff) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dword %2, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(dst), "v"(voff), "s"(rs), "s"(soff)
      : "memory");
}

// code value × block absmax, exact constants folded (0 → 0, ±1 → ±s: bit-identical to the product)
template <int I>
__device__ __forceinline__ float mulc(float s) {
  if constexpr (kNF4c[I] == 1.0f) return s;
  else if constexpr (kNF4c[I] == -1.0f) return -s;
  else if constexpr (kNF4c[I] == 0.0f) return 0.0f;
  else return vmul(s, kNF4c[I]);
}

// A lane's block table as byte planes (l[q] byte i = low byte of T[4q + i], h[q] the high bytes) and
// the expansion state of one 8-element chunk.  The expansion is cut into MICRO-OPS of at most two VALU
// instructions each, spread one per MFMA over the K-tile: a 16x16x32 MFMA holds the SIMD's issue for
// 8 of its 16 cycles, so two 4-cycle VALU fit beside it for free and a third does not
// (MI355X_MICROARCH.md, per-instruction constants; measured: 4-VALU micro-ops every ~2 MFMAs cost
// +31 % wave-cycles, profiles/r4/).
struct W4St {
  uint32_t l[4], h[4];
  float m0, m1, m2, m3;
  uint32_t p0, p1;
  uint32_t sa, sb, t4, w4, w8, w12, ma, mb, x0, x1, x2, x3, lo, hi;
  u32x4 o;
};
// entry I of a block's table: NF4 (MODE 1) code_I · absmax; affine int4 (MODE 2, W4A16 GPTQ / AWQ)
// (I − z)·s — exactly Int4Weight.dequantize's fp32 expression (I − z is exact)
template <int I, int MODE>
__device__ __forceinline__ float tab_entry(float s, float zf) {
  if constexpr (MODE == 2) return vmul(s, (float)I - zf);
  else return mulc<I>(s);
}
// table micro-op J (0..15): q = J / 4 builds planes l[q], h[q] from T[4q .. 4q+3]
template <int J, int MODE>
__device__ __forceinline__ void w4_table(W4St& t, float s, float zf) {
  constexpr int q = J / 4, r = J % 4;
  if constexpr (r == 0) {
    t.m0 = tab_entry<4 * q, MODE>(s, zf);
    t.m1 = tab_entry<4 * q + 1, MODE>(s, zf);
  } else if constexpr (r == 1) {
    t.p0 = pk_bf16(t.m0, t.m1);
    t.m2 = tab_entry<4 * q + 2, MODE>(s, zf);
  } else if constexpr (r == 2) {
    t.m3 = tab_entry<4 * q + 3, MODE>(s, zf);
    t.p1 = pk_bf16(t.m2, t.m3);
  } else {
    t.l[q] = vperm(t.p1, t.p0, 0x06040200u);
    t.h[q] = vperm(t.p1, t.p0, 0x07050301u);
  }
}
// chunk micro-op P (0..11) on the 8 codes in w (nibble b of byte j = element j + 4b):
//  0-1 selectors (low 3 bits of each code, one byte per element) and shifted copies of w;
//  2-3 masks 0xFF where code >= 8 (v_perm selectors 8..11 replicate bit 15 / 31 of either source);
//  4-7 elements 0-3: lo / hi plane lookups, select, interleave to bf16 pairs;  8-11 elements 4-7
template <int P>
__device__ __forceinline__ void w4_chunk(W4St& u, uint32_t w) {
  if constexpr (P == 0) {
    u.sa = w & 0x07070707u;
    u.t4 = w >> 4;
  } else if constexpr (P == 1) {
    u.sb = u.t4 & 0x07070707u;
    u.w4 = w << 4;
  } else if constexpr (P == 2) {
    u.w8 = w << 8;
    u.w12 = w << 12;
  } else if constexpr (P == 3) {
    u.ma = vperm(u.w12, u.w4, 0x090B080Au);
    u.mb = vperm(u.w8, w, 0x090B080Au);
  } else if constexpr (P == 4 || P == 8) {
    const uint32_t sel = P == 4 ? u.sa : u.sb;
    u.x0 = vperm(u.l[1], u.l[0], sel);
    u.x1 = vperm(u.l[3], u.l[2], sel);
  } else if constexpr (P == 5 || P == 9) {
    const uint32_t sel = P == 5 ? u.sa : u.sb;
    u.x2 = vperm(u.h[1], u.h[0], sel);
    u.x3 = vperm(u.h[3], u.h[2], sel);
  } else if constexpr (P == 6 || P == 10) {
    const uint32_t m = P == 6 ? u.ma : u.mb;
    u.lo = vbfi(m, u.x1, u.x0);
    u.hi = vbfi(m, u.x3, u.x2);
  } else {
    u.o[P == 7 ? 0 : 2] = vperm(u.hi, u.lo, 0x05010400u);
    u.o[P == 7 ? 1 : 3] = vperm(u.hi, u.lo, 0x07030602u);
  }
}

// EPI (fused MLP epilogues; SURVEY.md K5 "activation in the GEMM epilogue"):
//   1  SwiGLU forward on the gate|up projection (NT, no split).  B = W_gu [2F, K] as stored ([gate | up]
//      rows); the tile's B rows are gathered so that fragment pair (2c, 2c+1) of a wave is gate rows
//      16c'…+15 and the matching up rows — every lane then holds g and u of the same (m, col).  Writes
//      gu [M, 2F] in the [gate | up] layout (saved for backward) and h = silu(g)·u [M, F] to aux_out;
//      either store is skipped when its pointer is null (a checkpointed layer's first forward discards gu,
//      its recompute needs no h).  N = 2F (virtual columns).
//   2  SwiGLU backward fused into the down projection's dX (BT, no split): the GEMM tile is dh [M, F];
//      the epilogue reads g, u from aux = gu [M, 2F] and writes dgu = [dh·u·silu'(g) | dh·silu(g)].
//      N = F.
// Both round the GEMM result to bf16 first, exactly where the unfused path stores it.
// W4: Bv = g4w-packed NF4 codes of W ([N, K] when NT, [K, N] when BT, as W is stored), bscale =
// decoded fp32 absmax transposed, [cols(W) / 64][rows(W)].
// LoRA branches fused into the forward GEMM (LORA = true): y += xa·Bᵀ over the adapters'
// column ranges, as nks extra 32-deep MFMA K-steps on the tile's accumulators — before the bf16
// rounding, so the adapter term is exact to fp32 like the base product.  xa [M, 32·nks] bf16 holds
// s_b·D_b(x)·A_bᵀ of every branch b in its k-slot [kofs_b, kofs_b + r_b) (multiples of 8, zero elsewhere:
// lora_proj / lora_proj2 outputs); B_b [n_b, r_b] bf16 covers GEMM columns [c0_b, c0_b + n_b).  The
// fragments come straight from global memory (16 B per lane; the tile's xa rows and B rows are
// L2-resident).  The workgroups of tile row 0 also write B_bᵀ [r_b, n_b] for the backward's dy·B
// projection when bt_b is given.
template <int BMT, int BN, bool BT, bool SPLIT, int EPI, int W4, bool LORA = false>
__global__ __launch_bounds__(NT, 1) void gemm4w_k(const bf16* __restrict__ A, int lda, const void* __restrict__ Bv,
                                                  int ldb, const bf16* __restrict__ residual, void* __restrict__ out,
                                                  int M, int N, int K, int splits, const bf16* __restrict__ aux,
                                                  bf16* __restrict__ aux_out, int F, float* __restrict__ ws,
                                                  const float* __restrict__ bscale, const float* __restrict__ bzero,
                                                  const LoraEpi lx, const LoraDx ldx) {
  static_assert(W4 != 2 || (!BT && EPI == 0 && !LORA), "affine int4 (W4A16): the plain forward");
  static_assert(EPI == 0 || !SPLIT, "fused epilogues run on whole-K tiles");
  static_assert(!LORA || (EPI == 0 && !SPLIT), "LoRA epilogues: plain forward / dX, whole-K tiles");
  static_assert(EPI != 1 || !BT, "SwiGLU forward epilogue: NT only");
  static_assert(EPI != 2 || BT, "SwiGLU backward epilogue: the transposed-B dX only");
  static_assert(BMT == 256 || BMT == 128, "tile heights: 256, 128");
  static_assert(!W4 || BN != 192, "W4: tile widths 128, 256");
  constexpr int NA = BMT / 32;                 // a fragments per wave per K-half
  constexpr int NB = BN / 32;                  // b fragments per wave per K-half
  constexpr int IMG_AT = BMT * BK * 2;
  constexpr int IMG_B = BN * BK * 2;
  constexpr int STAGE = IMG_AT + IMG_B;
  constexpr int NLD = BN / 128;                // W4: 1 KB code DMAs per wave per K-tile
  constexpr int NSC = W4 == 2 ? 2 : 1;         // W4: per-block fp32 words per lane (absmax | scale, zero)
  constexpr int CR_W = NLD * 1024 + 256 * NSC; // W4: a wave's codes + tables of one K-tile (LDS ring)
  constexpr int RING = W4 ? 2 * 4 * CR_W : 0;  // W4: two K-tiles of codes in flight
  constexpr int STAGES = 3 * STAGE + RING <= 160 * 1024 ? 3 : 2;
  static_assert(BN == 128 || BN == 256 || (BN == 192 && !(BT && LORA)), "tile widths: 128, 256, 192 (not the LoRA dX)");
  constexpr int KT = 2 * NA * NB;              // MFMAs per K-tile per wave
  constexpr int H = KT / 2;
  constexpr int R = NA + NB;                   // fragment-read items per K-half
  constexpr int DA = BMT / 32;                 // A DMAs per wave per K-tile
  constexpr int DB = W4 ? 0 : BN / 32;         // B DMAs per wave per K-tile
  constexpr int D = DA + DB;                   // all DMAs per wave per K-tile
  constexpr int NCL = W4 ? NLD + NSC : 0;      // W4: LDS-DMAs per wave per K-tile for codes + tables
  constexpr int NCH = 4 * NLD;                 // W4: 8-element chunks a lane expands per K-tile
  constexpr int KV = D + NCL;                  // vector-memory instructions per wave per K-tile
  constexpr bool BIG = NA == 8;
  constexpr int K1 = R + (BIG ? 9 : 1);        // barrier 1 after this MFMA
  constexpr int K2 = KT - R - 1;               // barrier 2 after this MFMA
  constexpr int DSP = (K2 - (BIG ? 10 : 2) - (K1 + 1)) / D;   // DMA spacing
  static_assert(DSP >= 1, "schedule");
  // W4 micro-op stream: 16 table ops, then 12 per chunk, spread evenly over MFMAs [M0S, KT - 1): the
  // code DMAs of tile t + STAGES + 1 go on MFMAs 0 .. NCL-1, the wait + LDS reads of tile t + STAGES's
  // codes on MFMA SW, the first micro-op 3 MFMAs later (the reads' latency)
  constexpr int SW = NCL;
  constexpr int M0S = SW + 3;
  constexpr int NM = 16 + 12 * NCH;
  constexpr int SPAN = KT - 1 - M0S;
  static_assert(!W4 || M0S + (27 * SPAN) / NM > K1, "W4: the first chunk's ds_write must follow barrier 1");
  __shared__ __attribute__((aligned(16))) char lds[STAGES * STAGE + RING];

  const int tiles_m = (M + BMT - 1) / BMT, tiles_n = (N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n * splits;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int sp = id % splits;
  const int tid = id / splits;
  const int tm = tid % tiles_m, tn = tid / tiles_m;
  const int m0 = tm * BMT, n0 = tn * BN;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int wr = w >> 1, wc = w & 1;

  const int nk_all = K / BK;
  const int per = (nk_all + splits - 1) / splits;
  const int kt0 = sp * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);

  // ---- DMA sources (per-lane byte offsets; the K-tile step goes in the scalar offset)
  const rsrc_t rsa = make_rsrc(A, (uint64_t)((size_t)(M - 1) * lda + K) * 2);
  const rsrc_t rsb = W4 ? make_rsrc(Bv, (uint64_t)N * K / 2)
                        : BT ? make_rsrc(Bv, (uint64_t)((size_t)(K - 1) * ldb + N) * 2)
                             : make_rsrc(Bv, (uint64_t)((size_t)(N - 1) * ldb + K) * 2);
  uint32_t va[8], vb[8];   // (fixed sizes: a lambda capturing a template-sized local array drops the
                          // kernel's host-side instantiation — hipcc / clang, ROCm 7.2)
  {
    const int r8 = lane >> 3, c = (lane & 7) ^ (r8 & 6);
#pragma unroll
    for (int i = 0; i < DA; ++i) {   // A: wave w, DMA i → rows (BMT/4)·w + 8i + r8
      const int ra = min(m0 + w * (BMT / 4) + i * 8 + r8, M - 1);
      va[i] = ((uint32_t)ra * (uint32_t)lda + (uint32_t)(kt0 * BK + c * 8)) * 2u;
    }
    if constexpr (W4) {
    } else if constexpr (!BT) {
#pragma unroll
      for (int i = 0; i < DB; ++i) {   // B rows (BN/4)·w + 8i + r8
        int rb;
        if constexpr (EPI == 1) {   // tile row rt → gate row or up row of h-column block 16·(rt / 32)
          const int rt = w * (BN / 4) + i * 8 + r8;
          const int hr = min(tn * (BN / 2) + 16 * (rt >> 5) + (rt & 15), F - 1);
          rb = (rt & 16) ? F + hr : hr;
        } else {
          rb = min(n0 + w * (BN / 4) + i * 8 + r8, N - 1);
        }
        vb[i] = ((uint32_t)rb * (uint32_t)ldb + (uint32_t)(kt0 * BK + c * 8)) * 2u;
      }
    } else {
      // the lane's 16 B of the lane-linear BT image (k-rows of 2·BN bytes; wave w fills rows 16w .. 16w + 15,
      // DMA i the next 1 KB of them — at BN = 192 a piece spans 2 2/3 rows), fetched from the swizzled column
#pragma unroll
      for (int i = 0; i < DB; ++i) {
        const int b = w * (IMG_B / 4) + i * 1024 + lane * 16;
        const int kr = b / (2 * BN), ch = (b % (2 * BN)) / 16;
        const int cc = ch ^ (2 * bt_swz<BN>(kr));
        vb[i] = ((uint32_t)(kt0 * BK + kr) * (uint32_t)ldb + (uint32_t)(n0 + 8 * cc)) * 2u;
      }
    }
  }
  const uint32_t b_step = BT ? (uint32_t)BK * (uint32_t)ldb * 2u : (uint32_t)(BK * 2);

  // ---- W4: code / absmax DMA offsets and the LDS B-image chunk addresses of this lane's block
  uint32_t w4c[2] = {0u, 0u}, w4s = 0u, w4cstep = 0u, w4sstep = 0u;
  int w4o[8];
  rsrc_t rss = rsb, rsz = rsb;
  if constexpr (W4) {
    const int hh = BN == 256 ? 0 : lane >> 5;   // BN = 128: the two lane halves take the block's k-halves
    if constexpr (!BT) {   // lane = one W row (tile row rt) × the K-tile's 64 k: one quant block
      const int rt = BN == 256 ? w * 64 + lane : w * 32 + (lane & 31);
      int n;
      if constexpr (EPI == 1) {
        const int hr = min(tn * (BN / 2) + 16 * (rt >> 5) + (rt & 15), F - 1);
        n = (rt & 16) ? F + hr : hr;
      } else {
        n = min(n0 + rt, N - 1);
      }
      const int KBw = K / 64;
#pragma unroll
      for (int j = 0; j < NLD; ++j)
        w4c[j] = (uint32_t)((((n >> 6) * KBw + kt0) * 2 + (BN == 256 ? j : hh)) * 1024 + (n & 63) * 16);
      w4cstep = 2048u;
      w4s = (uint32_t)(kt0 * N + n) * 4u;
      w4sstep = (uint32_t)N * 4u;
      rss = make_rsrc(bscale, (uint64_t)N * (K / 64) * 4);
      if constexpr (W4 == 2) rsz = make_rsrc(bzero, (uint64_t)N * (K / 64) * 4);
      const int rl = rt - w * (BN / 4);   // row within the wave's BN/4 rows
#pragma unroll
      for (int u = 0; u < NCH; ++u)
        w4o[u] = IMG_AT + w * (IMG_B / 4) + (rl >> 3) * 1024 + 16 * slot_of<true>(rl & 7, 4 * hh + u);
    } else {   // lane = one W row (GEMM k-row kr of the tile) × 64 (or 32) W columns: one quant block
      const int kr = 16 * w + (lane & 15);
      const int cb = BN == 256 ? lane >> 4 : (lane >> 4) & 1;
      const int KBw = N / 64;
      const int kbw = min(n0 / 64 + cb, KBw - 1);
#pragma unroll
      for (int j = 0; j < NLD; ++j)
        w4c[j] = (uint32_t)(((kt0 * KBw + kbw) * 2 + (BN == 256 ? j : hh)) * 1024 + kr * 16);
      w4cstep = (uint32_t)KBw * 2048u;
      w4s = (uint32_t)(kbw * K + kt0 * 64 + kr) * 4u;
      w4sstep = 256u;
      rss = make_rsrc(bscale, (uint64_t)K * (N / 64) * 4);
      const int hk = bt_swz<BN>(kr);
#pragma unroll
      for (int u = 0; u < NCH; ++u) w4o[u] = IMG_AT + kr * (2 * BN) + 16 * ((8 * cb + 4 * hh + u) ^ (2 * hk));
    }
  }

  // ---- fragment read offsets
  int lo[2], lob[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    lo[s] = ((lane >> 3) & 1) * 1024 + 16 * slot_of<false>(lane & 7, 4 * s + (lane >> 4));
    lob[s] = ((lane >> 3) & 1) * 1024 + 16 * slot_of<(W4 != 0)>(lane & 7, 4 * s + (lane >> 4));
  }
  const int a_off = wr * NA * 2048;
  const int b_off = wc * NB * 2048;
  int boff_t[8];
  if constexpr (BT) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int hk = bt_swz<BN>(8 * g + q);   // = the swizzle of row + 4 and of the second K-half's rows
#pragma unroll
    for (int j = 0; j < NB; ++j)
      boff_t[j] = (8 * g + q) * (2 * BN) + 32 * ((wc * NB + j) ^ hk) + 16 * (p >> 1) + 8 * (p & 1);
  }

  f32x4 acc[8][8];   // [NA..7][NB..7] unused for the smaller tiles
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];

  // LDS-DMA as asm statements: hipcc then tracks no LDS-DMA and does not drain the whole queue
  // (vmcnt(0)) in front of the first ds_read_b64_tr_b16 of the next tile, which it cannot prove
  // disjoint from the in-flight stages (measured: the dX kernel waited 33 % of its cycles there).
  // Every ordering of DMA'd data is by the explicit vmcnt + barrier pairs below.
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)lds);
  const uint32_t wa = lds_base + (uint32_t)w * (IMG_AT / 4), wb = lds_base + IMG_AT + (uint32_t)w * (IMG_B / 4);
  auto dma_a = [&](uint32_t st, int t, int q) {
    dma_lds(rsa, wa + st + q * 1024, va[q], (uint32_t)t * (BK * 2));
  };
  auto dma_b = [&](uint32_t st, int t, int q) {
    dma_lds(rsb, wb + st + q * 1024, vb[q], (uint32_t)t * b_step);
  };
  auto dma_tile = [&](uint32_t st, int t) {
#pragma unroll
    for (int q = 0; q < DA; ++q) dma_a(st, t, q);
#pragma unroll
    for (int q = 0; q < DB; ++q) dma_b(st, t, q);
  };
  // read item r of K-half s of the stage at st into (fa, fb)
  auto read_item = [&](bf16x8* fa, bf16x8* fb, const char* st, int s, int r) {
    if (sched_of<NA, NB>().rd_a[r]) {
      fa[sched_of<NA, NB>().rd_i[r]] = lds_frag(st + a_off + sched_of<NA, NB>().rd_i[r] * 2048 + lo[s]);
    } else if constexpr (BT) {
      const char* pb = st + IMG_AT + s * (32 * 2 * BN) + boff_t[sched_of<NA, NB>().rd_i[r]];
      const bf16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)pb);
      const bf16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(pb + 4 * 2 * BN));
      fb[sched_of<NA, NB>().rd_i[r]] = bf16x8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    } else {
      fb[sched_of<NA, NB>().rd_i[r]] = lds_frag(st + IMG_AT + b_off + sched_of<NA, NB>().rd_i[r] * 2048 + lob[s]);
    }
  };

  // W4: the codes + absmax of tile X are LDS-DMA'd (asm, counted by the explicit vmcnt waits like the A
  // tiles) into ring slot X & 1 one K-tile before the tile that expands them reads them back — each lane
  // its own 16-B pieces and dword, so the wave's own vmcnt orders them (no barrier)
  const uint32_t ring = lds_base + STAGES * STAGE + (uint32_t)w * CR_W;
  auto dma_code_item = [&](int slot, int t, int i) {
    if (i < NLD) dma_lds(rsb, ring + slot * (4 * CR_W) + i * 1024, w4c[i], (uint32_t)t * w4cstep);
    else if (i == NLD) dma_lds4(rss, ring + slot * (4 * CR_W) + NLD * 1024, w4s, (uint32_t)t * w4sstep);
    else dma_lds4(rsz, ring + slot * (4 * CR_W) + NLD * 1024 + 256, w4s, (uint32_t)t * w4sstep);
  };
  auto dma_codes = [&](int slot, int t) {
#pragma unroll
    for (int i = 0; i < NCL; ++i) dma_code_item(slot, t, i);
  };
  u32x4 cq[2];
  float csc = 0.f, czf = 0.f;
  auto read_codes = [&](int slot) {
    const char* rp = lds + STAGES * STAGE + slot * (4 * CR_W) + w * CR_W;
#pragma unroll
    for (int j = 0; j < NLD; ++j) cq[j] = *reinterpret_cast<const u32x4*>(rp + j * 1024 + lane * 16);
    csc = *reinterpret_cast<const float*>(rp + NLD * 1024 + lane * 4);
    if constexpr (W4 == 2) czf = *reinterpret_cast<const float*>(rp + NLD * 1024 + 256 + lane * 4);
  };
  W4St st4;
  // micro-op J of the expansion of the codes in cq / csc into the stage at byte offset so
  auto w4_mop = [&](auto j_c, uint32_t so) {
    constexpr int J = decltype(j_c)::value;
    if constexpr (J < 16) {
      w4_table<J, W4>(st4, csc, czf);
    } else {
      constexpr int u = (J - 16) / 12, p = (J - 16) % 12;
      w4_chunk<p>(st4, cq[u / 4][u % 4]);
      if constexpr (p == 11) *reinterpret_cast<u32x4*>(lds + so + w4o[u]) = st4.o;
    }
  };
  auto w4_all = [&](uint32_t so) {
    Unroll<0, NM>::run([&](auto jc) { w4_mop(jc, so); });
  };

  if (nk <= 0) {
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
    // ---- LoRA terms, computed in the prologue (at the end of the tile they ran serialized — every tile of a
    // round finishes at once: +10-13 µs per call)
    //  NT: K-step 0 of the adapters' extra K (xa·Bᵀ) initialises the accumulators;
    //  BT: the masked input-gradient term Σ_b D_b(ds_b·g_b·A_b) initialises them.
    // Operands come by compiler-visible global loads, drained by vmcnt(0) BEFORE the first LDS-DMA is issued:
    // no counted wait ever guards a register load beside the DMAs (the round-5 dK/dV race:
    // profiles/r5/zero3_dkv_race.txt; pinned by tests/test_vmcnt_audit_cpu.py).  The loads hit L2 (xa / g were
    // written by the launch before), so the drain costs one L2 latency per workgroup.
    bf16x8 lxe[8], lbe[8], lbe2[8], lxe2[8];
    u32x4 lkeep[2][8], lga[2][8], lgb[2][8];
    if constexpr (LORA && !BT) {
      const int q = lane >> 4;   // 8-deep k-block of K-step 0
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int m = min(m0 + wr * (BMT / 2) + i * 16 + (lane & 15), M - 1);
        lxe[i] = *reinterpret_cast<const bf16x8*>((const bf16*)lx.xa + (size_t)m * lx.ldxa + 8 * q);
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int n = n0 + wc * (BN / 2) + j * 16 + (lane & 15);
        const bf16* src = (const bf16*)lx.xa;   // any valid address; masked below
        int hit = -1;
        for (int b = 0; b < lx.nbr; ++b) {
          const int kk = 8 * q - lx.kofs[b];
          if (n >= lx.c0[b] && n < lx.c0[b] + lx.n[b] && kk >= 0 && kk < lx.r[b]) {
            src = (const bf16*)lx.b[b] + (size_t)(n - lx.c0[b]) * lx.r[b] + kk;
            hit = b;
          }
        }
        lbe[j] = *reinterpret_cast<const bf16x8*>(src);
        lkeep[0][j][0] = (uint32_t)hit;
      }
      __builtin_amdgcn_s_waitcnt(WAIT_VM0);
    }
    if constexpr (LORA && BT) {
      constexpr int CPR = BN / 8;
      // A_b columns [n0, n0 + BN) as the k-rows 0..31 of a BT image per branch (LDS offset b·64·BN; rows >= r_b
      // zero), read back by the main loop's transposed reads; the LDS is free before the prologue DMAs
      for (int b = 0; b < ldx.nbr; ++b) {
        const bf16* Ab = (const bf16*)ldx.a[b];
        for (int idx = threadIdx.x; idx < 32 * CPR; idx += NT) {
          const int kr = idx / CPR, cc = idx % CPR;
          const int hk = bt_swz<BN>(kr);
          const int col = n0 + 8 * cc;
          bf16x8 v = {};
          if (kr < ldx.r[b] && col < N) v = *reinterpret_cast<const bf16x8*>(Ab + (size_t)kr * N + col);
          *reinterpret_cast<bf16x8*>(lds + b * (64 * BN) + kr * (2 * BN) + 16 * (cc ^ (2 * hk))) = v;
        }
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const bf16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(lds + boff_t[j]));
        const bf16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(lds + boff_t[j] + 4 * 2 * BN));
        lbe[j] = bf16x8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
        if (ldx.nbr > 1) {
          const bf16x4 y0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(lds + 64 * BN + boff_t[j]));
          const bf16x4 y1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(lds + 64 * BN + boff_t[j] + 4 * 2 * BN));
          lbe2[j] = bf16x8{y0[0], y0[1], y0[2], y0[3], y1[0], y1[1], y1[2], y1[3]};
        }
      }
      // g_b rows (fp32, 8 per lane: ranks 8·(lane/16) ..) and the keep bits of the lane's 16-byte run of
      // k (covers its NB 16-column blocks: 4 bits per block)
      const int kq = 8 * (lane >> 4);
      const int kb0 = ((n0 + wc * (BN / 2)) >> 3) & ~15;   // 16-B aligned keep-byte run (N % 128 == 0)
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int m = min(m0 + wr * (BMT / 2) + i * 16 + (lane & 15), M - 1);
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          if (b >= ldx.nbr) break;
          const float* gp = ldx.g[b] + (size_t)m * ldx.ldg + (kq < ldx.r[b] ? kq : 0);
          // keep bits: 16 B = the lane's row over [n0 + wc·BN/2, + 128) (BN/2 ≤ 128 columns)
          const unsigned char* kp = ldx.keep[b] + (size_t)m * (N >> 3) + min(kb0, (N >> 3) - 16);
          lga[b][i] = *reinterpret_cast<const u32x4*>(gp);
          lgb[b][i] = *reinterpret_cast<const u32x4*>(gp + 4);
          lkeep[b][i] = *reinterpret_cast<const u32x4*>(kp);
        }
      }
      __builtin_amdgcn_s_waitcnt(WAIT_VM0);
      __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
      __syncthreads();   // every wave has read the staged A images: the DMAs may overwrite them
    }

    // prologue: tiles 0 .. STAGES-1 (clamped: past the last tile the DMAs re-stage tile nk-1 into
    // stages nobody reads again), wait for tile 0, read its first half.  W4: the B images of those
    // tiles are expanded here first; then the vector-memory stream takes its steady-state order
    // (the codes of tile STAGES ahead of the A DMAs of tile STAGES-1) so every counted wait below holds.
    if constexpr (W4) {
#pragma unroll
      for (int s = 0; s < STAGES; ++s) {   // B images of tiles 0 .. STAGES-1, one at a time via ring slot 1
        dma_codes(1, min(s, nk - 1));
        wait_vmcnt<0>();
        read_codes(1);
        w4_all((uint32_t)(s * STAGE));
      }
#pragma unroll
      for (int s = 0; s < STAGES; ++s) {
        if (s == STAGES - 1) dma_codes(0, min(STAGES, nk - 1));
        dma_tile(s * STAGE, min(s, nk - 1));
      }
      wait_vmcnt<(STAGES - 1) * DA + NCL>();
      __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
    } else {
#pragma unroll
      for (int s = 0; s < STAGES; ++s) dma_tile(s * STAGE, min(s, nk - 1));
      wait_vmcnt<(STAGES - 1) * D>();
    }
    __builtin_amdgcn_s_barrier();
    if constexpr (LORA && !BT) {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int hit = (int)lkeep[0][j][0];
        if (hit < 0) lbe[j] = bf16x8{};
        else if (tm == 0 && lx.bt[hit] != nullptr) {   // Bᵀ [r_b, n_b] for the backward, once per column
          const int n = n0 + wc * (BN / 2) + j * 16 + (lane & 15);
          const int kk = 8 * (lane >> 4) - lx.kofs[hit];
#pragma unroll
          for (int e = 0; e < 8; ++e) ((bf16*)lx.bt[hit])[(size_t)(kk + e) * lx.n[hit] + (n - lx.c0[hit])] = lbe[j][e];
        }
      }
#pragma unroll
      for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) mfma_zero(acc[i][j], lbe[j], lxe[i]);
    }
    if constexpr (LORA && BT) {
      const int kq = 8 * (lane >> 4);
#pragma unroll
      for (int i = 0; i < NA; ++i) {
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          if (b >= ldx.nbr) break;
          bf16x8 a;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v = __builtin_bit_cast(float, e < 4 ? lga[b][i][e] : lgb[b][i][e - 4]);
            a[e] = kq + e < ldx.r[b] ? (bf16)v : (bf16)0.f;
          }
          (b ? lxe2[i] : lxe[i]) = a;
        }
      }
      const int sub = ((lane >> 4) & 1) * 4;   // the lane's 4 columns inside each 8-column keep byte
      const int kb0 = ((n0 + wc * (BN / 2)) >> 3) & ~15;
      const int rel = ((n0 + wc * (BN / 2)) >> 3) - min(kb0, (N >> 3) - 16);
#pragma unroll
      for (int i = 0; i < NA; ++i) {
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          f32x4 v = acc[i][j];
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            if (b >= ldx.nbr) break;
            const f32x4 t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b ? lbe2[j] : lbe[j], b ? lxe2[i] : lxe[i],
                                                                   f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            const u32x4 kw = b ? lkeep[1][i] : lkeep[0][i];
            const int byte = min(rel + 2 * j + (lane >> 5), 15);   // (16 j + 4 (lane>>4)) / 8 into the run
            const uint32_t bits = (kw[byte >> 2] >> (8 * (byte & 3) + sub)) & 15u;
            const float ds = ldx.ds[b];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += ((bits >> e) & 1u) ? t[e] * ds : 0.f;
          }
          acc[i][j] = v;
          asm volatile("" : "+a"(acc[i][j]));   // into the AGPRs here, not right before the first MFMA
        }
      }
      // the inline-asm MFMAs read acc as SrcC; the compiler's hazard checks do not see into them, so the
      // v_accvgpr_write → MFMA SrcC distance is padded by hand (without it the last-written lane of a
      // tile read a stale value: non-finite dX entries in every 4th column)
      asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    }
#pragma unroll
    for (int r = 0; r < R; ++r) read_item(fa0, fb0, lds, 0, r);

    int cur = 0;   // stage of tile t (byte offset)
    auto body = [&](auto first, int t) {
      const int tn_ = t + STAGES < nk ? t + STAGES : nk - 1;
      const int tc_ = t + STAGES + 1 < nk ? t + STAGES + 1 : nk - 1;
      char* const cs_ = lds + cur;
      char* const ns = lds + (cur + STAGE == STAGES * STAGE ? 0 : cur + STAGE);
      Unroll<0, KT>::run([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        constexpr int i = sched_of<NA, NB>().i[k % H], j = sched_of<NA, NB>().j[k % H];
        if constexpr (k < H) {
          if constexpr (decltype(first)::value) mfma_zero(acc[i][j], fb0[j], fa0[i]);
          else mfma_acc(acc[i][j], fb0[j], fa0[i]);
        } else {
          mfma_acc(acc[i][j], fb1[j], fa1[i]);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (k < R) read_item(fa1, fb1, cs_, 1, k);
        if constexpr (W4) {
          if constexpr (k < NCL) dma_code_item((t + 1) & 1, tc_, k);
          if constexpr (k == SW) {   // tile t + STAGES's codes (DMA'd one tile ago) have landed
            wait_vmcnt<DA + NCL>();
            read_codes(t & 1);
          }
          if constexpr (k >= M0S && k < M0S + SPAN) {
            // micro-ops J with M0S + J·SPAN/NM == k
            constexpr int jlo = ((k - M0S) * NM + SPAN - 1) / SPAN;
            constexpr int jhi = ((k - M0S + 1) * NM + SPAN - 1) / SPAN;
            Unroll<jlo, (jhi < NM ? jhi : NM)>::run([&](auto jc) { w4_mop(jc, (uint32_t)cur); });
          }
        }
        if constexpr (k == K1) {
          __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (k > K1 && (k - K1 - 1) % DSP == 0 && (k - K1 - 1) / DSP < D) {
          constexpr int d = (k - K1 - 1) / DSP;
          if constexpr (d < DA) dma_a(cur, tn_, d);
          else dma_b(cur, tn_, d - DA);
        }
        if constexpr (k == K2) {
          wait_vmcnt<(STAGES - 1) * KV>();
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (k > K2) read_item(fa0, fb0, ns, 0, k - K2 - 1);
        __builtin_amdgcn_sched_barrier(0);
      });
      cur = cur + STAGE == STAGES * STAGE ? 0 : cur + STAGE;
    };
    body(std::integral_constant<bool, !LORA>{}, 0);
    for (int t = 1; t < nk; ++t) body(std::integral_constant<bool, false>{}, t);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  }

  if constexpr (LORA && !BT) {   // K-steps 1 .. nks-1 of the adapters (step 0 ran in the prologue)
    const int kb = lane >> 4;
    if (lx.nks > 1) {
    for (int s = 1; s < lx.nks; ++s) {
      bf16x8 xe[8], be[8];
      const int q = 4 * s + kb;   // this lane's 8-deep k-block of the extra K
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int m = min(m0 + wr * (BMT / 2) + i * 16 + (lane & 15), M - 1);
        xe[i] = *reinterpret_cast<const bf16x8*>((const bf16*)lx.xa + (size_t)m * lx.ldxa + 8 * q);
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int n = n0 + wc * (BN / 2) + j * 16 + (lane & 15);
        bf16x8 v = {};
        for (int b = 0; b < lx.nbr; ++b) {
          const int kk = 8 * q - lx.kofs[b];
          if (n >= lx.c0[b] && n < lx.c0[b] + lx.n[b] && kk >= 0 && kk < lx.r[b]) {
            v = *reinterpret_cast<const bf16x8*>((const bf16*)lx.b[b] + (size_t)(n - lx.c0[b]) * lx.r[b] + kk);
            if (tm == 0 && lx.bt[b] != nullptr) {   // Bᵀ [r_b, n_b] for the backward, once per column
#pragma unroll
              for (int e = 0; e < 8; ++e) ((bf16*)lx.bt[b])[(size_t)(kk + e) * lx.n[b] + (n - lx.c0[b])] = v[e];
            }
          }
        }
        be[j] = v;
      }
#pragma unroll
      for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) mfma_acc(acc[i][j], be[j], xe[i]);
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 2" ::: "memory");   // MFMA results → AGPR reads below
    }
  }

  // ---- epilogue: lane holds C[m = col][n = 4·(lane>>4) + r … +3] of each 16×16 block
  if constexpr (EPI == 1) {
    // h-block hb = gate block 2hb + up block 2hb + 1 (the gathered B rows); h-blocks paired for 16-B stores
    constexpr int NH = NB / 2;
    const int r4 = lane >> 4;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int m = m0 + wr * (BMT / 2) + i * 16 + (lane & 15);
      if (m >= M) continue;
#pragma unroll
      for (int hp = 0; hp + 1 < NH; hp += 2) {
        f32x4 g0 = acc[i][2 * hp], g1 = acc[i][2 * hp + 2], u0 = acc[i][2 * hp + 1], u1 = acc[i][2 * hp + 3];
        pair_swap(g0, g1);
        pair_swap(u0, u1);
        const int hc = tn * (BN / 2) + 16 * (wc * NH + hp + (r4 & 1)) + 8 * (r4 >> 1);
        if (hc >= F) continue;
        bf16x8 g, u, h;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          g[e] = (bf16)(e < 4 ? g0[e] : g1[e - 4]);
          u[e] = (bf16)(e < 4 ? u0[e] : u1[e - 4]);
          h[e] = (bf16)(silu_f((float)g[e]) * (float)u[e]);
        }
        if (out != nullptr) {
          bf16* gu = reinterpret_cast<bf16*>(out) + (size_t)m * 2 * F + hc;
          G4W_ST(reinterpret_cast<bf16x8*>(gu), g);
          G4W_ST(reinterpret_cast<bf16x8*>(gu + F), u);
        }
        if (aux_out != nullptr) G4W_ST(reinterpret_cast<bf16x8*>(aux_out + (size_t)m * F + hc), h);
      }
      if constexpr (NH % 2) {   // the unpaired last h-block (BN = 192): 8-B stores
        constexpr int j = NB - 2;
        const int hc = tn * (BN / 2) + 16 * (wc * NH + j / 2) + 4 * r4;
        if (hc < F) {
          bf16x4 g, u, h;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            g[e] = (bf16)acc[i][j][e];
            u[e] = (bf16)acc[i][j + 1][e];
            h[e] = (bf16)(silu_f((float)g[e]) * (float)u[e]);
          }
          if (out != nullptr) {
            bf16* gu = reinterpret_cast<bf16*>(out) + (size_t)m * 2 * F + hc;
            G4W_ST(reinterpret_cast<bf16x4*>(gu), g);
            G4W_ST(reinterpret_cast<bf16x4*>(gu + F), u);
          }
          if (aux_out != nullptr) G4W_ST(reinterpret_cast<bf16x4*>(aux_out + (size_t)m * F + hc), h);
        }
      }
    }
    return;
  }
  if constexpr (SPLIT) {   // fp32 slab of this split; splitk_sum_k adds the slabs (+ residual)
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int m = m0 + wr * (BMT / 2) + i * 16 + (lane & 15);
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int n = n0 + wc * (BN / 2) + j * 16 + 4 * (lane >> 4);
        if (n < N) G4W_ST(reinterpret_cast<f32x4*>(ws + ((size_t)sp * M + m) * N + n), acc[i][j]);
      }
    }
    return;
  }
  // Epilogues that read global memory (residual; EPI 2's g / u) issue every load of four accumulator
  // rows before the first use, from clamped (always valid) addresses — one latency per four rows, not
  // one per 16×16 block (a load behind a per-block bounds branch waits vmcnt(0) each time).  Blocks are
  // paired (pair_swap) so every load and store moves 16 B per lane.
  const bool has_res = EPI == 0 && residual != nullptr;
  constexpr int RC = 4;   // rows per chunk (NA is 4 or 8: a multiple)
  constexpr int NP = NB / 2;   // block pairs per row (NB is even)
  const int r4 = lane >> 4;
  auto rows = [&](auto hh_c, auto res_c) {
    constexpr int i0 = RC * decltype(hh_c)::value;
    constexpr bool RES = decltype(res_c)::value;
    bf16x8 la[RC][4], lb[RC][4];
#pragma unroll
    for (int ii = 0; ii < RC; ++ii) {
      const int m = min(m0 + wr * (BMT / 2) + (i0 + ii) * 16 + (lane & 15), M - 1);
#pragma unroll
      for (int jp = 0; jp < NP; ++jp) {
        const int n = min(n0 + wc * (BN / 2) + 16 * (2 * jp + (r4 & 1)) + 8 * (r4 >> 1), N - 8);
        if constexpr (EPI == 2) {
          const bf16* gp = aux + (size_t)m * 2 * F + n;
          la[ii][jp] = *reinterpret_cast<const bf16x8*>(gp);
          lb[ii][jp] = *reinterpret_cast<const bf16x8*>(gp + F);
        } else if constexpr (RES) {
          la[ii][jp] = *reinterpret_cast<const bf16x8*>(residual + (size_t)m * N + n);
        }
      }
    }
#pragma unroll
    for (int ii = 0; ii < RC; ++ii) {
      const int m = m0 + wr * (BMT / 2) + (i0 + ii) * 16 + (lane & 15);
      if (m >= M) continue;
#pragma unroll
      for (int jp = 0; jp < NP; ++jp) {
        // (the swap partners, lanes r and r ^ 1 of one row, must both be active: swap before the column check;
        // the row check above is uniform across partners — they share m)
        f32x4 a = acc[i0 + ii][2 * jp], b = acc[i0 + ii][2 * jp + 1];
        pair_swap(a, b);
        const int n = n0 + wc * (BN / 2) + 16 * (2 * jp + (r4 & 1)) + 8 * (r4 >> 1);
        if (n >= N) continue;
        if constexpr (EPI == 2) {
          bf16x8 dg, du;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = (float)(bf16)(e < 4 ? a[e] : b[e - 4]), g = (float)la[ii][jp][e], uu = (float)lb[ii][jp][e];
            const float sg = 1.f / (1.f + __expf(-g));
            du[e] = (bf16)(d * (g * sg));
            dg[e] = (bf16)(d * uu * (sg * (1.f + g * (1.f - sg))));
          }
          bf16* dp = reinterpret_cast<bf16*>(out) + (size_t)m * 2 * F + n;
          G4W_ST(reinterpret_cast<bf16x8*>(dp), dg);
          G4W_ST(reinterpret_cast<bf16x8*>(dp + F), du);
        } else {
          bf16x8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float x = e < 4 ? a[e] : b[e - 4];
            o[e] = (bf16)(RES ? x + (float)la[ii][jp][e] : x);
          }
          G4W_ST(reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(out) + (size_t)m * N + n), o);
        }
      }
    }
  };
  if (has_res) {
    Unroll<0, NA / RC>::run([&](auto hc) { rows(hc, std::true_type{}); });
  } else {
    Unroll<0, NA / RC>::run([&](auto hc) { rows(hc, std::false_type{}); });
  }
}

inline int tiles_of(int M, int N, int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); }

}  // namespace
