// mgn_diag.h -- diagnostic builds only (tools/build_variant.py passes
// -DMGN_DIAG): the cycle stamps, iteration stamps and wall-clock records of
// the step kernels, and the ablation switches, which produce wrong outputs
// and exist to time what a part of the step costs.  In the product build
// every hook below is empty, and setting an ablation or stamp macro without
// MGN_DIAG is an error.
#pragma once

#if !defined(MGN_DIAG) &&                                                                            \
    (defined(MGN_STAMPS) || defined(MGN_WALLX) || defined(MGN_ITERSTAMP) || defined(MGN_ABL_NOSTORE) ||  \
     defined(MGN_ABL_NOSTORE_ASSET) || defined(MGN_ABL_NOSTORE_ENV) || defined(MGN_ABL_DRAW) ||          \
     defined(MGN_TRIO_ABL_PRO) || defined(MGN_TRIO_ABL_G) || defined(MGN_TRIO_ABL_L) ||                  \
     defined(MGN_TRIO_ABL_F) || defined(MGN_TRIO_ABL_EPI) || defined(MGN_NST_ABL_TERM) ||                \
     defined(MGN_NST_ABL_SUM) || defined(MGN_NST_ABL_ROW) || defined(MGN_NO_GK))
#error "stamp / ablation switches belong to diagnostic builds (-DMGN_DIAG, tools/build_variant.py)"
#endif

namespace mgn {

// The diagnostic switches as the step kernels read them: MGN_ST(...) is code
// of the stamp builds only (it names the stamp buffers, which exist only
// there); kAbl* are the ablation builds' switches, false in every product
// build, so a product kernel reads straight through `if constexpr` blocks
// that the compiler discards.
#ifdef MGN_STAMPS
#define MGN_ST(...) __VA_ARGS__
#else
#define MGN_ST(...)
#endif
#ifdef MGN_TRIO_ABL_PRO
constexpr bool kAblPro = true;   // no state loads
#else
constexpr bool kAblPro = false;
#endif
#ifdef MGN_TRIO_ABL_G
constexpr bool kAblG = true;     // no tick (prices frozen)
#else
constexpr bool kAblG = false;
#endif
#ifdef MGN_TRIO_ABL_L
constexpr bool kAblL = true;     // no Broker orders
#else
constexpr bool kAblL = false;
#endif
#ifdef MGN_TRIO_ABL_F
constexpr bool kAblF = true;     // no step finish, no outputs
#else
constexpr bool kAblF = false;
#endif
#ifdef MGN_TRIO_ABL_EPI
constexpr bool kAblEpi = true;   // no state write-back
#else
constexpr bool kAblEpi = false;
#endif
#ifdef MGN_NST_ABL_TERM
constexpr bool kAblNstTerm = true;  // no n-step summand arithmetic
#else
constexpr bool kAblNstTerm = false;
#endif
#ifdef MGN_NST_ABL_SUM
constexpr bool kAblNstSum = true;   // no n-step ordered sum
#else
constexpr bool kAblNstSum = false;
#endif
#ifdef MGN_NST_ABL_ROW
constexpr bool kAblNstRow = true;   // no zero entries of the n-step rows
#else
constexpr bool kAblNstRow = false;
#endif
#ifdef MGN_ABL_NOSTORE_ASSET
constexpr bool kAblNoStoreAsset = true;  // no per-asset output stores
#else
constexpr bool kAblNoStoreAsset = false;
#endif
#ifdef MGN_ABL_NOSTORE_ENV
constexpr bool kAblNoStoreEnv = true;    // no per-env output stores
#else
constexpr bool kAblNoStoreEnv = false;
#endif

#ifdef MGN_STAMPS
// diagnostic build only: per role, cycles of [work 1, wait A, work 2, wait B]
// summed over one wave per role and block, then the iteration count
__device__ unsigned long long g_duo_stamps[24];
// per-block sub-phase accumulators, one writer (the block's first ledger lane)
__shared__ unsigned long long s_duo_sub[8];
// wall clock (s_memrealtime, 100 MHz) per block (first 2048 blocks), plain
// stores by one lane: [0] generator entry, [1] ledger entry, [2] ledger loop
// start, [3] ledger loop end, [4] generator loop end, [5] generator exit,
// [6] / [7] ledger after iteration 0 / 2
__device__ unsigned long long g_duo_wall[2048 * 32];
#define MGN_T(v) v = __builtin_amdgcn_s_memtime()
#define MGN_WALL(i) if ((threadIdx.x & 255) == 0 && blockIdx.x < 2048) g_duo_wall[blockIdx.x * 32 + (i)] = __builtin_amdgcn_s_memrealtime()
#elif defined(MGN_WALLX)
// lighter diagnostic build: the wall stamps, the hardware ids and per block
// the slowest iteration's phases ([12] generator store phase, [13] its
// iteration, [14] ledger phase 1, [15] its iteration), no cycle accumulators
__device__ unsigned long long g_duo_stamps[24];
__device__ unsigned long long g_duo_wall[2048 * 32];
#define MGN_T(v)
#define MGN_WALL(i) if ((threadIdx.x & 255) == 0 && blockIdx.x < 2048) g_duo_wall[blockIdx.x * 32 + (i)] = __builtin_amdgcn_s_memrealtime()
#else
#define MGN_T(v)
#define MGN_WALL(i)
#endif
#ifdef MGN_WALLX
#define MGN_RT(v) v = __builtin_amdgcn_s_memrealtime()
#define MGN_WALLV(i, val_) if ((threadIdx.x & 255) == 0 && blockIdx.x < 2048) g_duo_wall[blockIdx.x * 32 + (i)] = (val_)
#else
#define MGN_RT(v)
#define MGN_WALLV(i, val_)
#endif

#ifdef MGN_ITERSTAMP
// diagnostic build: s_memtime stamps of the first 256 blocks, 64 slots each --
// [0] entry, [1] after the prologue barrier, [2 + j] generator lane 0 after
// iteration j's barrier (j < 40), [44] generator / [45] ledger / [46] finish
// lane 0 after its epilogue stores (with their completion wait); [47] G lane 0
// once the kernel arguments arrived, [48] G lane 0 once its iteration-0 tick
// is published to LDS, [49] L lane 0 once its iteration-0 records are
// published, [50] F lane 0 once its iteration-1 outputs are issued; [51] L
// state loaded, [52] / [53] L's orders start / done (iteration 0), [54] G
// state loaded, [55] / [56] / [57] F's iteration-1 sums / reward / shaping
// done, [58] L's prevEq formed (iteration 0)
__device__ unsigned long long g_iter[256 * 64];
#define MGN_IT(slot, lane0)                                             \
  if (threadIdx.x == (lane0) && blockIdx.x < 256 && (slot) < 64)        \
    g_iter[blockIdx.x * 64 + (slot)] = __builtin_amdgcn_s_memtime()
#define MGN_IT_DRAIN() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#else
#define MGN_IT(slot, lane0)
#define MGN_IT_DRAIN()
#endif


}  // namespace mgn
