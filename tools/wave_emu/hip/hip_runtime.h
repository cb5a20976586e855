// Host shim used ONLY by tools/wave_emu: lets csrc/tmg_board.hip compile with
// g++ so each wavefront runs as 64 user-space fibers (one OS thread), for
// AddressSanitizer / gdb.  Lanes run one after another between collectives
// (ballot, readlane, fences/barriers), which are resolved once every lane of
// the wave has arrived — the lockstep points of the real wavefront.
#pragma once
#include <stdint.h>
#include <cstdlib>

#define __device__
#define __host__
#define __global__
#define __launch_bounds__(...)
#define __align__(x) alignas(x)
#define __forceinline__ inline
#define __shared__

struct EmuDim { unsigned x = 0, y = 0, z = 0; };
EmuDim emu_thread_idx();
extern EmuDim emu_block_idx, emu_grid_dim;
#define threadIdx (emu_thread_idx())
#define blockIdx (emu_block_idx)
#define gridDim (emu_grid_dim)

enum EmuOp { EMU_SYNC = 1, EMU_BALLOT = 2, EMU_READLANE = 3, EMU_DPP = 4 };
// lane side of a collective: publish (op, value, arg), yield to the scheduler,
// return the resolved result
uint64_t emu_collective(int op, uint64_t v, int arg);
unsigned char *emu_smem();

inline void emu_sync() { emu_collective(EMU_SYNC, 0, 0); }
inline uint64_t __ballot(int pred) { return emu_collective(EMU_BALLOT, pred ? 1 : 0, 0); }
inline uint32_t emu_readlane(uint32_t v, int l) { return (uint32_t)emu_collective(EMU_READLANE, v, l); }
inline uint32_t emu_readfirstlane(uint32_t v) { return emu_readlane(v, 0); }
inline int emu_readfirstlane(int v) { return (int)emu_readlane((uint32_t)v, 0); }
// DPP: arg packs ctrl | row_mask << 12 | bank_mask << 16 | bound_ctrl << 20; value packs old << 32 | src
inline int emu_update_dpp(int old, int src, int ctrl, int row_mask, int bank_mask, bool bound_ctrl) {
    uint64_t v = ((uint64_t)(uint32_t)old << 32) | (uint32_t)src;
    return (int)(uint32_t)emu_collective(EMU_DPP, v, ctrl | (row_mask << 12) | (bank_mask << 16) | ((bound_ctrl ? 1 : 0) << 20));
}
#define __builtin_amdgcn_update_dpp(o, s, c, r, b, bc) emu_update_dpp((o), (s), (c), (r), (b), (bc))
// the builtin returns int (an OR into a 64-bit value sign-extends it, as on the device)
#define __builtin_amdgcn_readlane(v, l) ((int)emu_readlane((uint32_t)(v), (l)))
#define __builtin_amdgcn_readfirstlane(v) ((int)emu_readlane((uint32_t)(v), 0))
#define __builtin_amdgcn_ds_bpermute(a, v) ((int)emu_readlane((uint32_t)(v), ((a) >> 2) & 63))
#define __builtin_amdgcn_alignbyte(a, b, s) \
    ((uint32_t)(((((uint64_t)(uint32_t)(a)) << 32) | (uint32_t)(b)) >> (8 * ((s) & 3))))
#define __builtin_amdgcn_alignbit(a, b, s) \
    ((uint32_t)(((((uint64_t)(uint32_t)(a)) << 32) | (uint32_t)(b)) >> ((s) & 31)))
#define __builtin_amdgcn_fence(order, scope) emu_sync()
#define __builtin_amdgcn_wave_barrier() ((void)0)
inline void __syncthreads() { emu_sync(); }
inline int __popcll(uint64_t x) { return __builtin_popcountll(x); }
inline int __clzll(uint64_t x) { return x ? __builtin_clzll(x) : 64; }
inline int __ffsll(unsigned long long x) { return __builtin_ffsll((long long)x); }
inline uint64_t __umul64hi(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) >> 64); }

struct alignas(16) uint4 { uint32_t x, y, z, w; };
inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return uint4{x, y, z, w}; }

inline int min(int a, int b) { return a < b ? a : b; }
inline int max(int a, int b) { return a > b ? a : b; }
inline unsigned min(unsigned a, unsigned b) { return a < b ? a : b; }
inline unsigned max(unsigned a, unsigned b) { return a > b ? a : b; }

inline uint64_t __builtin_amdgcn_s_memrealtime() { return 0; }
inline unsigned atomicAdd(unsigned *p, unsigned v) { unsigned o = *p; *p += v; return o; }
inline unsigned long long atomicAdd(unsigned long long *p, unsigned long long v) { unsigned long long o = *p; *p += v; return o; }
// lanes run one at a time between collectives, so a plain read-modify-write is the atomic
inline unsigned long long atomicOr(unsigned long long *p, unsigned long long v) { unsigned long long o = *p; *p |= v; return o; }
inline void __threadfence() {}

inline unsigned emu_mbcnt_lo(unsigned m, unsigned acc) {
    const unsigned l = emu_thread_idx().x;
    return acc + (unsigned)__builtin_popcount(m & (l >= 32 ? 0xffffffffu : ((1u << l) - 1u)));
}
inline unsigned emu_mbcnt_hi(unsigned m, unsigned acc) {
    const unsigned l = emu_thread_idx().x;
    return acc + (unsigned)__builtin_popcount(m & (l <= 32 ? 0u : ((1u << (l - 32)) - 1u)));
}
#define __builtin_amdgcn_mbcnt_lo(m, a) emu_mbcnt_lo((m), (a))
#define __builtin_amdgcn_mbcnt_hi(m, a) emu_mbcnt_hi((m), (a))
#define __builtin_amdgcn_s_setprio(p) ((void)0)
#define TMG_OPAQUE_V(x) ((void)0)

#define TMG_CONST_AS
#define TMG_KEEP_V3(x, y, z) ((void)0)
#define TMG_KEEP_V(x) ((void)0)
#define TMG_SMEM_DECL(name) unsigned char *name = emu_smem()
#define TMG_KERNARG_PARAMS(p) (p)
