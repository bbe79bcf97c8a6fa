// ghost_amd — shared device helpers for the gfx950 (MI355X / CDNA4) kernels.
//
// Activations are NHWC ("pixel-major, channel-contiguous") so that
//   * every conv is an implicit GEMM whose K dimension (tap, channel) is contiguous,
//   * the AAD mask (a dot product over channels per pixel) is a contiguous reduction,
//   * 1x1 convs on z_attr are plain row-major GEMMs.
// A channel stride `ld` (elements between consecutive pixels) lets producers write
// straight into a channel slice of a wider buffer (the unet skip concat, the fused
// x/h' concat of AAD_ResBlk) with no copy.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

// A/B tuning knobs.  Only a tuning build (GHOST_TUNING=1 python -m ghost_amd.build, which adds
// -DGHOST_TUNING) reads them from the environment; the shipping library compiles each knob to the
// default that the measurements chose, so no process-global switch changes its behaviour.
#ifdef GHOST_TUNING
inline int ghost_env_knob(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
#define GHOST_KNOB(name, dflt) ghost_env_knob(name, dflt)
#else
#define GHOST_KNOB(name, dflt) (dflt)
#endif

#define GHOST_DEV __device__ __forceinline__

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

enum GhostDType { GHOST_F32 = 0, GHOST_BF16 = 1, GHOST_F16 = 2, GHOST_U8 = 3 };

// Last-arriver reductions (split-K fix-up, InstanceNorm final pass): the partials one workgroup hands to another
// cross XCDs, whose L2s are not coherent with each other.  The hand-off is MI355X_MICROARCH.md's producer form
// "{sc1 stores} -> every storing wave's s_waitcnt vmcnt(0) -> workgroup barrier -> one lane's agent-scope atomic
// add" and its consumer form "the workgroup whose add came last -> ONE agent acquire -> s_waitcnt vmcnt(0) ->
// __syncthreads() -> loads", which the guide validates at any number of workgroups per CU (its sc1-loads-only
// variant without the acquire is validated at one workgroup per CU only, and in_stats_partial_kernel /
// conv_igemm_kernel run several).  Only the last arriver pays the acquire (one L1 invalidate of its CU); a
// release / acquire fence in EVERY producing workgroup (each writes back or invalidates its XCD's L2) made the
// fused GEMMs 2-6x slower than the GEMM + reduction kernel pair they replace.
// Every write of a handed-off partial MUST be st_dev (a write-through sc1 store), and every read of one ld_dev:
// a plain store would sit in the producer XCD's L2, which the consumer's acquire does not reach.
// The sc1 lowering of these accesses is the gfx94x / gfx950 memory model's; the library is built for gfx950 only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "ghost_amd kernels target gfx950 only (last_arrival's hand-off relies on gfx950's sc1 write-through lowering)"
#endif
GHOST_DEV void st_dev(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
GHOST_DEV float ld_dev(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// this workgroup's arrival at *cnt after its st_dev stores (every thread calls it; 1-D workgroups): true in the
// last of n arrivals, which also resets the counter for the next launch on the stream and acquires the other
// workgroups' partials for its CU before any thread reads them.  `flag` is a word of the kernel's own LDS array,
// free at this point: a second __shared__ object beside an LDS-DMA ring makes hipcc wait vmcnt(0) before the first
// LDS read of every K step (cdna_hip_programming.md §6 item 4a; measured here: the split GEMMs' ring drained every
// step, +1.8 us per B = 1 GEMM).  The caller must not overwrite `flag` before a barrier.
GHOST_DEV bool last_arrival(unsigned* cnt, unsigned n, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's device-scope stores acknowledged
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = old == n - 1;
    if (old == n - 1) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // buffer_inv sc1: this CU's L1
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the invalidate has completed before the barrier
    }
  }
  __syncthreads();
  return *flag != 0;
}

GHOST_DEV float to_f(float v) { return v; }
GHOST_DEV float to_f(bf16 v) { return (float)v; }
GHOST_DEV float to_f(_Float16 v) { return (float)v; }
GHOST_DEV float to_f(uint8_t v) { return (float)v; }

template <typename T> GHOST_DEV T from_f(float v);
template <> GHOST_DEV float from_f<float>(float v) { return v; }
template <> GHOST_DEV bf16 from_f<bf16>(float v) { return (bf16)v; }
template <> GHOST_DEV _Float16 from_f<_Float16>(float v) { return (_Float16)v; }

// elements per 16-byte vector
template <typename T> struct Vec16 { static constexpr int N = 16 / sizeof(T); };

// load / store VEC elements (16 bytes) converting to / from fp32
template <typename T> GHOST_DEV void load16_f(const T* p, float* out) {
  u32x4 raw = *reinterpret_cast<const u32x4*>(p);
  const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
  for (int i = 0; i < Vec16<T>::N; ++i) out[i] = to_f(e[i]);
}
template <typename T> GHOST_DEV void store16_f(T* p, const float* in) {
  u32x4 raw;
  T* e = reinterpret_cast<T*>(&raw);
#pragma unroll
  for (int i = 0; i < Vec16<T>::N; ++i) e[i] = from_f<T>(in[i]);
  *reinterpret_cast<u32x4*>(p) = raw;
}

// the same with a non-temporal (streaming) store: for a large output that is not read again before it
// has left the caches
template <typename T> GHOST_DEV void store16_f_nt(T* p, const float* in) {
  u32x4 raw;
  T* e = reinterpret_cast<T*>(&raw);
#pragma unroll
  for (int i = 0; i < Vec16<T>::N; ++i) e[i] = from_f<T>(in[i]);
  __builtin_nontemporal_store(raw, reinterpret_cast<u32x4*>(p));
}

GHOST_DEV float sigmoidf_ref(float x) { return 1.0f / (1.0f + expf(-x)); }
// v_exp_f32 + v_rcp_f32 (a few ulp from sigmoidf_ref): for masks blended into bf16 outputs
GHOST_DEV float sigmoid_fast(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

// packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two lanes' worth of fp32 per instruction)
typedef __attribute__((ext_vector_type(2))) float f32x2;
GHOST_DEV f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
// the two bf16 of a 32-bit word (element 0 in the low half) as fp32
GHOST_DEV f32x2 bf16x2_f(unsigned w) { return f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)}; }

// ---- 16-bit storage types: bf16 (the throughput path) and fp16 (a .half() module, the reference's GPU
// precision).  Kernels that store activations in 16 bits are templated on the storage type T and use these
// helpers for everything type-specific: the 8-element MFMA operand, the MFMA itself (both run at the same
// rate on gfx950), and unpacking the two values of a 32-bit word to fp32.
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
template <typename T> struct V8;
template <> struct V8<bf16> { typedef bf16x8 t; };
template <> struct V8<_Float16> { typedef f16x8 t; };
template <typename T> using v8_t = typename V8<T>::t;

template <typename T> GHOST_DEV f32x4 mfma16x16x32(v8_t<T> a, v8_t<T> b, f32x4 c);
template <> GHOST_DEV f32x4 mfma16x16x32<bf16>(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <> GHOST_DEV f32x4 mfma16x16x32<_Float16>(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// the two 16-bit values of a 32-bit word (element 0 in the low half) as fp32
template <typename T> GHOST_DEV f32x2 unpack2(unsigned w);
template <> GHOST_DEV f32x2 unpack2<bf16>(unsigned w) { return bf16x2_f(w); }
template <> GHOST_DEV f32x2 unpack2<_Float16>(unsigned w) {
  typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
  const f16x2 h = __builtin_bit_cast(f16x2, w);
  return f32x2{(float)h.x, (float)h.y};
}
// two fp32 -> one 32-bit word of T (round to nearest even, as (T)v)
template <typename T> GHOST_DEV unsigned pack2(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) T t2;
  // one vector conversion: a single v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32 (two scalar casts became two
  // conversions and a v_perm_b32)
  const t2 v = __builtin_convertvector(f32x2{a, b}, t2);
  return __builtin_bit_cast(unsigned, v);
}

// relu of two fp32 values rounded to T and packed: round first (v_cvt_pk_*), then one packed max on the
// 16-bit halves — rounding keeps the sign, so relu(round(v)) == round(relu(v)).  bf16 as signed int16: every
// negative value (and -0) is a negative integer, so max(x, 0) zeroes exactly those (v_pk_max_i16); fp16 with
// v_pk_max_f16.
template <typename T> GHOST_DEV unsigned relu_pack2(f32x2 v);
template <> GHOST_DEV unsigned relu_pack2<bf16>(f32x2 v) {
  typedef __attribute__((ext_vector_type(2))) short s16x2;
  const s16x2 x = __builtin_bit_cast(s16x2, pack2<bf16>(v.x, v.y));
  return __builtin_bit_cast(unsigned, __builtin_elementwise_max(x, s16x2{0, 0}));
}
template <> GHOST_DEV unsigned relu_pack2<_Float16>(f32x2 v) {
  typedef __attribute__((ext_vector_type(2))) short s16x2;
  // fp16 as signed int16 orders the same way as bf16 (sign-magnitude with the sign in bit 15)
  const s16x2 x = __builtin_bit_cast(s16x2, pack2<_Float16>(v.x, v.y));
  return __builtin_bit_cast(unsigned, __builtin_elementwise_max(x, s16x2{0, 0}));
}

// Whole-row stores of a 16-pixel x 64-channel 16-bit tile held as MFMA epilogues hold it: lane (lr, lq) has ow0 =
// 16-byte chunk m (channels 8 m .. 8 m + 7, m in 0..3 set by lq) and ow1 = chunk 4 + m of pixel lr.  One exchange
// between lanes lr and lr ^ 8 (DPP row_ror:8, by bank mask) and the first store writes pixels 0-7 (lane: pixel lr & 7,
// chunk m + 4 (lr >> 3)), the second pixels 8-15: each store instruction writes 8 whole 128-byte rows instead of 16
// half rows.  The half-row form took 1.4-1.7x the time of its bytes (B = 64 AADBlk7 pair: 240.5 -> 174.5 us, the
// same kernel with the stores skipped 115 us; profiles/r04_ab_aad_stores.txt).
// o + pa / o + pb: the channel-0 element of the lane's pixel lr & 7 / 8 + (lr & 7).
template <typename T>
GHOST_DEV void store_rows16(T* __restrict__ o, long pa, long pb, int lr, int m, const u32x4& ow0, const u32x4& ow1) {
  u32x4 rA, rB;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    // row_ror:8 = 0x128; bank mask 0xC: lanes 8-15 of each 16-lane row take their partner's value, 0x3: lanes 0-7
    rA[k] = (unsigned)__builtin_amdgcn_update_dpp((int)ow0[k], (int)ow1[k], 0x128, 0xF, 0xC, false);
    rB[k] = (unsigned)__builtin_amdgcn_update_dpp((int)ow1[k], (int)ow0[k], 0x128, 0xF, 0x3, false);
  }
  const int c = (m + 4 * (lr >> 3)) * 8;
  *reinterpret_cast<u32x4*>(o + pa + c) = rA;
  *reinterpret_cast<u32x4*>(o + pb + c) = rB;
}

// ghost dtype enum of a storage type
template <typename T> constexpr int gdt();
template <> constexpr int gdt<float>() { return GHOST_F32; }
template <> constexpr int gdt<bf16>() { return GHOST_BF16; }
template <> constexpr int gdt<_Float16>() { return GHOST_F16; }
inline bool is16(int dt) { return dt == GHOST_BF16 || dt == GHOST_F16; }

// workgroup id -> work index such that each XCD (the hardware deals workgroups round-robin over the
// 8 XCDs) gets one contiguous run of work indices, so neighbours that share input lines hit the same
// L2 (cdna_hip_programming.md T1, bijective form)
GHOST_DEV int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  const int xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// shuffle-xor reduction over `width` lanes (width power of two, <= 64)
GHOST_DEV float group_sum(float v, int width) {
  for (int o = width >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
