// MI355X (gfx950) content-defined chunking kernels.
//
// Replaces the per-byte FastCDC Gear loop of ext go-cdc-chunkers v0.0.8
// chunkers/fastcdc (*FastCDC).Algorithm and the (*Chunker).Next driver loop
// consumed at plakar snapshot/backup.go:647-665.  See DESIGN.md for the data
// layout and the roofline of each kernel.
//
// Pipeline per launch group (<= 32 independent buffers):
//   k_scan2     the byte scan.  Every lane rolls the Gear fingerprint
//               over its own run (512 B - 8 KiB, sized so the launch fills
//               every CU; 64-byte warm-up: the masked bits only
//               depend on the last W <= 64 bytes), tests MaskS at every
//               position and appends the rare hits to a candidate index of
//               64-KiB blocks (u16 offsets).
//   k_resolve   the chain of cuts, one wave per resolution segment, in one
//               launch: a speculative chain from the segment start (walked
//               through a successor graph of the segment's candidates built
//               lane-parallel in LDS), the junction from the previous
//               segment's speculative exit, a decoupled look-back for the
//               true entry and the cut offset, then the cut list and the
//               result row.  Pathological data (and the debug mode) fall back
//               to a sequential single-wave walk of the buffer.
//
// next(p) is wave-cooperative and decides exactly what the reference decides:
// the truncated window [p+Min, p+Min+W-1) (fingerprint reset at p+Min) by a
// 64-lane weighted prefix scan, full-window MaskS hits from the index, and the
// MaskL region [p+Normal, p+n) by an on-demand raw wave scan.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <type_traits>
#include <vector>

#include "cdc_internal.h"

namespace cdc {

// s_sleep count (64 cycles each) between polls of a look-back or ticket wait
#ifndef CDC_SPIN_SLEEP
#define CDC_SPIN_SLEEP 1
#endif
constexpr int kSpinSleep = CDC_SPIN_SLEEP;

static constexpr uint64_t kNoHit = ~0ull;
static constexpr uint32_t kRawLaneBytes = 512;  // bytes tested per lane per raw-scan block (C3 +5-8 % over 256)
static constexpr uint32_t kWarm = 64;           // warm-up bytes (>= W - 1 for any mask)

// ---------------------------------------------------------------------------
// Gear table in LDS: 256 entries x 32 copies, 256 B per entry.  Lane l reads
// copy (l & 31), so the 32 lanes of a ds_read_b64 lane group always hit 32
// distinct bank pairs: conflict-free gathers whatever the data bytes are.
// Byte address of entry b for this lane = (b << 8) | ((lane & 31) << 3),
// built from the packed data word by one v_perm_b32.
// ---------------------------------------------------------------------------
// NT threads fill a COPIES-copy table (entry e, copy c at index COPIES e + c),
// optionally in the scan's shifted frame.  Any NT: the 256 * COPIES slots are
// strided over the block (the global loads of the 2-KiB table hit L2 / L1).
// The walkers use 8 copies (16 KiB; they are latency-bound and tolerate a few
// bank conflicts), so a walker workgroup fits beside a scan workgroup on a CU.
template <int NT, int COPIES = 32>
__device__ __forceinline__ void fill_gear_lds(uint64_t *tab, const uint64_t *gear, uint32_t sh = 0)
{
    static_assert(NT % 64 == 0, "block size");
    constexpr uint32_t kSlots = 256u * COPIES;
    constexpr int kPer = int((kSlots + NT - 1) / NT);
    uint64_t v[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const uint32_t x = threadIdx.x + uint32_t(i) * NT;
        v[i] = x < kSlots ? gear[x / COPIES] : 0;
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const uint32_t x = threadIdx.x + uint32_t(i) * NT;
        if (x < kSlots) tab[x] = v[i] << sh;
    }
}
// Walker table copies: 8 by default (16 KiB).  32 (the scan's layout:
// conflict-free gathers, one-instruction v_perm address) made C3's raw MaskL
// scans 3.5 % faster but C1 2 % slower (a 64-KiB fill per walker workgroup).
constexpr uint32_t kWCopies = 8;
constexpr uint32_t kWEntShift = kWCopies == 32 ? 8 : kWCopies == 16 ? 7 : 6;  // log2(kWCopies * 8)
static_assert(kWCopies == 8 || kWCopies == 16 || kWCopies == 32, "walker table copies");

__device__ __forceinline__ uint64_t lds_gear(const char *tab, uint32_t addr)
{
    return *reinterpret_cast<const uint64_t *>(tab + addr);
}

// Address-space-typed views for code the compiler does not inline into its
// kernel (next_node and what it calls): there a generic pointer becomes flat
// loads, which count in both vmcnt and lgkmcnt, so each LDS wait also waits
// for the global loads in flight (and LDS reads through flat are slower).
typedef __attribute__((address_space(3))) const char lds_char;
typedef __attribute__((address_space(1))) const uint64_t g_u64;
typedef __attribute__((address_space(1))) const uint32_t g_u32;
typedef __attribute__((address_space(1))) const uint8_t g_u8;

__device__ __forceinline__ uint64_t lds_gear(const lds_char *tab, uint32_t addr)
{
    return *reinterpret_cast<__attribute__((address_space(3))) const uint64_t *>(tab + addr);
}

template <typename T>
__device__ __forceinline__ T *as_space(uint64_t addr)  // an address as a typed pointer
{
    return reinterpret_cast<T *>(uintptr_t(addr));
}

__device__ __forceinline__ const lds_char *as_lds(const char *p)  // LDS offset of a generic LDS pointer
{
    return as_space<const lds_char>(uint32_t(reinterpret_cast<uintptr_t>(p)));
}

// 16 bytes at a 16-B aligned global address (two 8-byte global loads).
__device__ __forceinline__ uint4 gload16(uint64_t a)
{
    const g_u64 *q = as_space<const g_u64>(a);
    const uint64_t x = q[0], y = q[1];
    return make_uint4(uint32_t(x), uint32_t(x >> 32), uint32_t(y), uint32_t(y >> 32));
}

__device__ __forceinline__ uint32_t gear_addr(uint32_t laneoff, uint32_t word, int k)
{
    // v_perm_b32: byte0 <- laneoff.byte0 (sel 4), byte1 <- word.byte(k), bytes 2,3 <- 0 (sel 0x0C)
    return __builtin_amdgcn_perm(laneoff, word, 0x0C0C0004u | (uint32_t(k & 3) << 8));
}

// Walker table address of byte k of word: (byte << kWEntShift) | ((lane & 7) << 3).
template <uint32_t ESH = kWEntShift>
__device__ __forceinline__ uint32_t wgear_addr(uint32_t wlaneoff, uint32_t word, int k)
{
    if constexpr (ESH == 8) return gear_addr(wlaneoff, word, k);  // 256-B entries: one v_perm
    return (__builtin_amdgcn_ubfe(word, uint32_t(k & 3) * 8u, 8u) << ESH) | wlaneoff;
}

__device__ __forceinline__ uint32_t key_of(uint64_t fp, uint32_t mlo, uint32_t mhi)
{
    // zero iff (fp & mask) == 0: (hi & mhi) | (lo & mlo) in two VALU
    return __builtin_amdgcn_bitop3_b32(uint32_t(fp >> 32), mhi, uint32_t(fp) & mlo, 0xEA);
}

__device__ __forceinline__ uint32_t word_of(const uint4 &d, int i)
{
    return i == 0 ? d.x : i == 1 ? d.y : i == 2 ? d.z : d.w;
}

__device__ __forceinline__ uint32_t umin3(uint32_t a, uint32_t b, uint32_t c)
{
    uint32_t r;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Roll 16 bytes and return the min of the 16 keys (0 iff some position hit).
// (Reducing the keys with v_min3 after the roll instead was 5 % slower on C3:
// the keys stay live across the chain.)
template <uint32_t ESH = kWEntShift, typename TP>
__device__ __forceinline__ uint32_t roll16_test(const uint4 &d, uint64_t &fp, TP tab,
                                                uint32_t laneoff, uint32_t mlo, uint32_t mhi)
{
    uint32_t acc = 0xFFFFFFFFu;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        fp = (fp << 1) + lds_gear(tab, wgear_addr<ESH>(laneoff, word_of(d, k >> 2), k));
        acc = min(acc, key_of(fp, mlo, mhi));
    }
    return acc;
}

template <uint32_t ESH = kWEntShift, typename TP>
__device__ __forceinline__ void roll16(const uint4 &d, uint64_t &fp, TP tab,
                                       uint32_t laneoff)
{
#pragma unroll
    for (int k = 0; k < 16; ++k)
        fp = (fp << 1) + lds_gear(tab, wgear_addr<ESH>(laneoff, word_of(d, k >> 2), k));
}

// General 16-byte group at absolute address a: positions < fz have fp = 0
// (the reference resets fp at p+Min), positions in [ts, te) are tested.
// Returns the first hit (absolute) or kNoHit; fp is advanced over the group.
template <uint32_t ESH = kWEntShift, typename TP>
__device__ __forceinline__ uint64_t group_first_hit(const uint4 &d, uint64_t &fp, uint64_t a,
                                                    uint64_t ts, uint64_t te, uint64_t fz,
                                                    TP tab, uint32_t laneoff,
                                                    uint32_t mlo, uint32_t mhi)
{
    uint64_t hit = kNoHit;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint64_t pos = a + k;
        const uint64_t g = lds_gear(tab, wgear_addr<ESH>(laneoff, word_of(d, k >> 2), k));
        fp = pos < fz ? 0ull : (fp << 1) + g;
        if (hit == kNoHit && pos >= ts && pos < te && pos >= fz && key_of(fp, mlo, mhi) == 0)
            hit = pos;
    }
    return hit;
}


// Copy a uniform value into a VGPR the compiler cannot fold back into an SGPR
// operand (VOP2 forms with a VGPR mask issue faster than with an SGPR one).
__device__ __forceinline__ uint32_t to_vgpr(uint32_t x)
{
    uint32_t v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(x));
    return v;
}

// ---------------------------------------------------------------------------
// Debug timestamps (B.debug & kDbgTs): s_memrealtime (100 MHz) at phase
// boundaries, read back with cdc_debug_timestamps().  Off in production.
// ---------------------------------------------------------------------------
constexpr uint32_t kDbgTs = 16;
constexpr uint32_t kDbgGraph = 32;  // with kDbgTs: k_resolve slots 5-7 time graph_build's phases
constexpr uint32_t kTsScan = 0;                       // 4 per scan workgroup (<= 4096)
constexpr uint32_t kTsRes = kTsScan + 4 * 4096;       // 8 per resolution segment (<= 16384)
constexpr uint32_t kTsClk = kTsRes + 8 * 16384;     // clock ring (B.debug & kDbgClk): 4 per scan launch
constexpr uint32_t kClkRecs = 4096;
constexpr uint32_t kTsClkN = kTsClk + 4 * kClkRecs;   // ring counter
constexpr uint32_t kTsHw = kTsClkN + 1;               // per scan workgroup: XCC_ID << 32 | HW_ID (kDbgTs)
constexpr uint32_t kTsAbort = kTsHw + 4096;           // the last wait that gave up: kind, two values, time
constexpr uint32_t kTsSlots = kTsAbort + 4;
constexpr uint32_t kDbgClk = 64;
__device__ uint64_t g_ts[kTsSlots];

__device__ __forceinline__ void dbg_ts(const Batch &B, uint32_t slot, uint64_t v = ~0ull)
{
    if ((B.debug & kDbgTs) && slot < kTsSlots) g_ts[slot] = v == ~0ull ? __builtin_amdgcn_s_memrealtime() : v;
}

// Bounded waits.  Every spin of a walker (granules, look-back statuses)
// gives up after the launch's spin limit of its own waiting (s_memrealtime,
// 100 MHz; W.flags[kLimitWord], written by the scan kernel: 2 s, or B.spin_ticks
// in the forced-abort debug mode) or as soon as another wait of the launch
// gave up.  It raises the launch's abort word (W.flags[kAbortWord]) and
// records what it waited for at g_ts[kTsAbort]; the wave then publishes an
// ABORTED status (look-back propagates it) and stores CDC_E_DEVICE into every
// result row of the launch group, so the caller gets an error instead of a
// hung device.  No correct launch waits that long.
constexpr uint32_t kAbortWord = kMaxBufsPerLaunch;
constexpr uint32_t kLimitWord = kMaxBufsPerLaunch + 1;  // spin limit, in 100-MHz ticks (>= 1)
constexpr uint64_t kSpinLimit = 200000000ull;            // 2 s
enum : uint32_t { kWaitJunction = 2, kWaitPrev, kWaitLook, kWaitLookSlow, kWaitLast };

struct SpinGuard {
    uint64_t t0 = 0, lim = 0;
    // true: poll again; false: give up
    __device__ __forceinline__ bool ok(uint32_t *flags, uint32_t kind, uint64_t a, uint64_t b)
    {
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (!t0) {
            t0 = now;
            lim = __hip_atomic_load(flags + kLimitWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (!lim) lim = kSpinLimit;
            return true;
        }
        if (__hip_atomic_load(flags + kAbortWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
        if (now - t0 < lim) return true;
        if ((threadIdx.x & 63u) == 0) {
            __hip_atomic_store(flags + kAbortWord, kind, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            g_ts[kTsAbort] = kind;
            g_ts[kTsAbort + 1] = a;
            g_ts[kTsAbort + 2] = b;
            g_ts[kTsAbort + 3] = now;
        }
        return false;
    }
};

// ---------------------------------------------------------------------------
// k_scan: the byte scan.  Each wave owns 64 lane runs of B.scan_lane bytes
// and stages them through one 4-KiB LDS slot per wave with LDS-DMA
// (global_load_lds_dwordx4, 4 per stage of 64 B per lane): pair staging,
// described at scan_body.
//
// The fingerprint runs in a shifted frame: the LDS Gear table holds
// G[b] << sh with sh = 63 - (highest MaskS bit), so fp' = fp << sh keeps every
// fp bit the masks can see (bits 0..hb) and the high dword of fp' holds the
// top 32 of them.  The hot test per byte is one v_and of that dword with the
// shifted MaskS high half (13 of the 15 default MaskS bits): a necessary
// condition, reduced by v_min3 to one wave-uniform branch per 32 bytes.  A
// lane whose filter fired (2^-13 per byte at the default masks: some lane of
// the wave in ~22 % of 32-byte groups) queues the group in LDS, and the queue
// is re-rolled exactly -- all mask bits, the run's bounds -- one group per
// lane, at the end of the task (see the recheck queue in scan_task), so
// warm-up bytes, bytes past the lane's run and lanes past the buffer's end
// need no separate code path: every stage of every lane runs the same
// straight-line loop.
//
// The next group's 16 Gear gathers are issued byte by byte between the links
// of the current group's fingerprint chain, into the registers its roll has
// just consumed.
//
// DMA addressing: one wave-uniform 64-bit base (SGPR pair) and one 32-bit
// per-lane offset per piece, the base advanced per stage; a wave whose pieces
// could leave the buffer clamps them to the buffer's last 16-byte block, so
// the warm-up before byte 0 and the ragged end read in-bounds bytes that the
// exact recheck then ignores.
// ---------------------------------------------------------------------------

#ifndef CDC_SCAN_WAVES
#define CDC_SCAN_WAVES 12
#endif
constexpr uint32_t kS2Waves = CDC_SCAN_WAVES;         // waves per scan workgroup (one workgroup per CU)
constexpr uint32_t kStage = 64;                       // bytes per lane per stage
constexpr uint32_t kL = kStage / 16;                  // 16-B pieces per lane per stage = DMAs per stage
constexpr uint32_t kGroups = kStage / 16;             // 16-byte groups per stage
constexpr uint32_t kStageBytes = 64u * kStage;        // per wave per stage (one LDS slot)
constexpr uint32_t kGearLdsBytes = 256u * 32u * 8u;   // 64 KiB
// Recheck queue: 32-byte groups per wave, 12 bytes each (fp before the group;
// its offset in the run and the lane).  64 items keep the scan workgroup at
// 121 KiB of LDS, so a k_resolve workgroup (36.3 KiB) of the other stream
// still fits beside it on a CU (at 128 items of 16 B it did not: pipelined
// -2 % warm, profiles/r06_*).
constexpr uint32_t kQCap = 64;
constexpr uint32_t kQBytes = kQCap * 12u;
// k_scan_f's recheck table: the Gear table in the MaskS frame, one copy (2 KiB)
constexpr uint32_t kFlushTabBytes = 256u * 8u;
static_assert(kGearLdsBytes + kS2Waves * (kStageBytes + kQBytes) + kFlushTabBytes + 37128u <= 160u * 1024u,
              "LDS budget: a scan workgroup and a k_resolve workgroup per CU");
// Scan lane lengths are multiples of kLaneQuant (16-B aligned runs: every lane
// of a buffer has the same stage alignment; 256 B avoided the slow strides
// seen at odd multiples of 128 B, see make_plan).
constexpr uint32_t kLaneQuant = 256;

template <int N>
__device__ __forceinline__ void wait_vmcnt()
{
    static_assert(N == 0, "vmcnt");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// One stage's kL LDS-DMA pieces in ONE asm statement: M0 is written and read
// inside it (and restored), every VGPR offset is read before the statement
// ends (trailing s_nop guards the compiler's next write of those registers).
// The staging loads are nontemporal (nt): the bytes are read once.  Measured
// (tools/ubench_pattern.hip, profiles/r05_scan_dma_nt_ab.txt): LDS-DMA of the
// scan's pattern reads 7.09 TB/s with nt against 6.20 without; the scan itself
// +4 % warm, +2 % under the driver's command.  CDC_SCAN_DMA_DEFAULT_POLICY
// builds the default-policy form (A/B only).
#ifdef CDC_SCAN_DMA_DEFAULT_POLICY
#define DMA_PIECE(i) "global_load_lds_dwordx4 %" #i ", %[base]\n\t"
#else
#define DMA_PIECE(i) "global_load_lds_dwordx4 %" #i ", %[base] nt\n\t"
#endif
#define DMA_NEXT "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
__device__ __forceinline__ void dma_stage(uint64_t base_in, uint32_t dst_in, const uint32_t (&off)[kL])
{
    static_assert(kL == 4, "four 1-KiB pieces per stage");
    // wave-uniform operands pinned to SGPRs (under VGPR pressure the compiler
    // may otherwise keep them in VGPRs, which the "s" constraint does not stop);
    // the statement opens with s_nop 4 (VALU-written SGPR read as a VMEM base)
    const uint64_t base = (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(base_in >> 32)))) << 32) |
                          uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(base_in)));
    const uint32_t dst = __builtin_amdgcn_readfirstlane(dst_in);
    uint32_t keep;
    asm volatile("s_nop 4\n\ts_mov_b32 %[keep], m0\n\ts_mov_b32 m0, %[dst]\n\ts_nop 0\n\t"
                 DMA_PIECE(1) DMA_NEXT DMA_PIECE(2) DMA_NEXT DMA_PIECE(3) DMA_NEXT DMA_PIECE(4)
                 "s_mov_b32 m0, %[keep]\n\ts_nop 1"
                 : [keep] "=&s"(keep)
                 : "v"(off[0]), "v"(off[1]), "v"(off[2]), "v"(off[3]), [base] "s"(base), [dst] "s"(dst)
                 : "memory", "scc");
}

// The same four pieces with M0 set once: piece j carries the instruction
// offset 1024 j, which LDS-DMA applies to the global AND the LDS address, so
// the per-lane offsets come with 1024 j already subtracted (offi) and M0 is
// not stepped between the pieces (3 SALU per stage fewer).
#ifdef CDC_SCAN_DMA_DEFAULT_POLICY
#define DMA_PIECE_IMM(i, o) "global_load_lds_dwordx4 %" #i ", %[base] offset:" #o "\n\t"
#else
#define DMA_PIECE_IMM(i, o) "global_load_lds_dwordx4 %" #i ", %[base] offset:" #o " nt\n\t"
#endif
__device__ __forceinline__ void dma_stage_imm(uint64_t base_in, uint32_t dst_in, const uint32_t (&offi)[kL])
{
    static_assert(kL == 4, "four 1-KiB pieces per stage");
    const uint64_t base = (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(base_in >> 32)))) << 32) |
                          uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(base_in)));
    const uint32_t dst = __builtin_amdgcn_readfirstlane(dst_in);
    uint32_t keep;
    asm volatile("s_nop 4\n\ts_mov_b32 %[keep], m0\n\ts_mov_b32 m0, %[dst]\n\ts_nop 0\n\t"
                 DMA_PIECE_IMM(1, 0) DMA_PIECE_IMM(2, 1024) DMA_PIECE_IMM(3, 2048) DMA_PIECE_IMM(4, 3072)
                 "s_mov_b32 m0, %[keep]\n\ts_nop 1"
                 : [keep] "=&s"(keep)
                 : "v"(offi[0]), "v"(offi[1]), "v"(offi[2]), "v"(offi[3]), [base] "s"(base), [dst] "s"(dst)
                 : "memory");
}

// One ticket per wave from an agent-scope counter.  Every lane takes part in
// the atomic (lane 0 adds 1, the others 0), so no lane-0 branch precedes the
// readfirstlane: after such a branch the compiler may thread it into a
// neighbouring lane-0 branch (round 5's one-launch resolver stored a flag
// there before its next claim), and the readfirstlane then runs for lanes 1-63
// while lane 0 is still on the other path -- they read 0 and loop on task 0
// (measured: a hang).
__device__ __forceinline__ uint32_t wave_ticket(uint32_t *p)
{
    const uint32_t old = __hip_atomic_fetch_add(p, (threadIdx.x & 63u) == 0u ? 1u : 0u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_readfirstlane(old);
}

__device__ __forceinline__ uint32_t scan_wave_max(uint32_t v)
{
#pragma unroll
    for (int o = 32; o; o >>= 1) v = max(v, uint32_t(__shfl_xor(int(v), o)));
    return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ uint32_t rec_cnt(uint64_t rec) { return uint32_t(rec & ((1u << kRecCntBits) - 1)); }
__device__ __forceinline__ uint32_t rec_ent(uint64_t rec, uint32_t e)
{
    return uint32_t(rec >> (kRecCntBits + kRecEntBits * e)) & ((1u << kRecEntBits) - 1);
}

// Each lane keeps its run's index record in a register (count + the first
// kRunCap offsets, see cdc_internal.h) and stores it after its last stage:
// one coalesced 8-byte store per run, no atomics.
__device__ __forceinline__ void record_hit(uint64_t &rec, int32_t r)
{
    const uint32_t c = rec_cnt(rec);
    if (c < kRunCap) rec |= uint64_t(uint32_t(r)) << (kRecCntBits + kRecEntBits * c);
    if (c < (1u << kRecCntBits) - 1) ++rec;
}

// Does scan task `t` of buffer D (buffer-relative) need the MaskL index?  A
// walker queries MaskL candidates from x0 = p + Normal only when the chunk start p found no full-window MaskS
// candidate in [p + Min + W - 1, p + Normal): a MaskS-free interval of
// Normal - Min - W + 1 bytes, holding at least kc complete MaskS index runs
// with no candidate.  In MaskS-run units, with [a, b) the maximal empty
// stretch holding those runs, x0 lies in runs a + kc .. b (run b, the first
// non-empty one, may hold x0 before its first candidate), and the search then
// runs to the first MaskL candidate past x0.  So a run r needs the index if
// r >= a + kc - 1 inside such a stretch, or if r <= b + kMaskLSpill after
// one; a longer search past the spill raw-scans.  The test reads the MaskS
// run records from kc + spill runs before the task to its end (256 per round
// trip) and decides each 64-run word with one lane per run and one ballot.
// It only decides where the index is built: a walker that
// finds no index for a task raw-scans it, so results never depend on it.
constexpr uint64_t kMaskLSpill = 16;  // MaskS runs after a long stretch's end (64: -1 %, 160: -11 % on C3)

__device__ bool maskl_needed(const Batch &B, const DevParams &P, const Workspace &W, const BufDesc &D, uint64_t t,
                             uint32_t lane)
{
    const uint64_t sl = B.scan_lane, tb = 64ull * sl;
    const uint64_t start = t * tb, end = min(D.len, start + tb);
    const uint64_t ra = start / sl, rb = (end - 1) / sl;  // the task's runs
    const uint64_t gap = P.normal_size - P.min_size - (P.win - 1);
    const uint32_t kc = uint32_t(gap / sl > 2 ? gap / sl - 1 : 1);
    const uint64_t r_lo = ra > kc + kMaskLSpill ? ra - kc - kMaskLSpill : 0;
    const uint64_t *runs = W.runs + 64ull * D.task_base;
    uint32_t cur = 0;  // empty runs ending just before the current word
    for (uint64_t r4 = r_lo; r4 <= rb; r4 += 256) {
        uint64_t rec[4];  // four words of records in flight: one round trip per 256 runs
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t q = r4 + 64u * j + lane;
            rec[j] = q <= rb ? runs[q] : 1ull;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t r0 = r4 + 64u * j;
            if (r0 > rb) break;
            const uint64_t E = __ballot(rec_cnt(rec[j]) == 0);
            const uint32_t n = uint32_t(min(rb + 1 - r0, uint64_t(64)));
            // Lane i looks at run r = r0 + i: the empty stretch ending at
            // r - 1 has `prev` runs (from the word's non-empty runs Z below
            // i, or cur + i when there are none).  An empty run needs the
            // index once its stretch reaches kc; a non-empty run after a long
            // stretch is that stretch's end b, which makes [b, b + spill]
            // need it.
            const uint64_t Z = ~E & (n == 64 ? ~0ull : (1ull << n) - 1);
            const uint64_t below = Z & ((1ull << lane) - 1);
            const uint32_t prev = below ? lane - 1u - (63u - uint32_t(__builtin_clzll(below))) : cur + lane;
            const uint64_t r = r0 + lane;
            bool need = false;
            if (lane < n) {
                if ((E >> lane) & 1ull)
                    need = r >= ra && prev + 1 >= kc;
                else
                    need = prev >= kc && r + kMaskLSpill >= ra;  // r <= rb holds
            }
            if (__ballot(need)) return true;
            cur = Z ? n - 1u - (63u - uint32_t(__builtin_clzll(Z))) : cur + n;
        }
    }
    return false;
}

template <bool kMaskL, bool kFused>
__device__ __forceinline__ void scan_task(const Batch &B, const DevParams &P, const Workspace &W, char *s_lds,
                                          const char *tab, uint32_t task, uint32_t lane, uint32_t wave,
                                          uint32_t laneoff);

// The byte scan.  kMaskL = false: the MaskS candidate index of every run
// (k_scan).  kMaskL = true: the MaskL index (k_scan_l), built only for the
// tasks maskl_needed() selects; every wave records validL for its task.
template <bool kMaskL, bool kFused = false>
__device__ __forceinline__ void scan_body(const Batch &B, const DevParams &P, const Workspace &W)
{
    static_assert(!(kMaskL && kFused), "k_scan_f builds both indexes, from the MaskS records' side");
    __shared__ __attribute__((aligned(16)))
    char s_lds[kGearLdsBytes + kS2Waves * (kStageBytes + kQBytes) + (kFused ? kFlushTabBytes : 0u)];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t laneoff = (lane & 31u) << 3;
    const uint32_t task = blockIdx.x * kS2Waves + wave;
    bool act = true;
    if constexpr (kMaskL) {
        act = false;
        if (task < B.total_tasks) {
            uint32_t bb = 0;
            while (bb + 1 < B.nbufs && task >= B.b[bb + 1].task_base) ++bb;
            const BufDesc &Db = B.b[bb];
            const uint64_t t = task - Db.task_base;
            if (t * 64ull * B.scan_lane < Db.len) act = maskl_needed(B, P, W, Db, t, lane);
            if (lane == 0) W.validL[task] = act ? 1u : 0u;
        }
        if (!__syncthreads_or(act ? 1 : 0)) return;  // no wave of this workgroup builds the index
        if (threadIdx.x == 0 && B.maskl_hint)
            __hip_atomic_store(B.maskl_hint, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if constexpr (!kMaskL) {  // k_resolve's per-segment status words and tickets of this launch group
        const uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
        for (uint32_t i = gt; i < B.total_segs; i += nth) {
            W.xg[i] = 0ull;
            W.sg[i] = 0ull;
        }
        if (gt < kMaxBufsPerLaunch + 4)  // + the abort word and the spin limit
            W.flags[gt] = gt == kLimitWord ? uint32_t(B.spin_ticks ? B.spin_ticks : kSpinLimit) : 0u;
        if (gt < 2) W.tick[gt] = 0u;
        if (gt < B.nbufs) B.b[gt].res->status = kRowPending;  // k_resolve's last segment settles it
        if (threadIdx.x == 0) dbg_ts(B, kTsScan + 4 * blockIdx.x);
    }
    // clock ring: workgroup 0's span in the 100-MHz and the shader-clock counters
    uint32_t clk = 0;
    if (!kMaskL && (B.debug & kDbgClk) && blockIdx.x == 0 && threadIdx.x == 0) {
        clk = kTsClk + 4u * uint32_t(atomicAdd(reinterpret_cast<unsigned long long *>(&g_ts[kTsClkN]), 1ull) % kClkRecs);
        g_ts[clk] = __builtin_amdgcn_s_memrealtime();
        g_ts[clk + 1] = __builtin_amdgcn_s_memtime();
    }
    fill_gear_lds<kS2Waves * 64>(reinterpret_cast<uint64_t *>(s_lds), W.gear,
                                 kFused ? P.fm_sh : kMaskL ? P.fl_sh : P.fs_sh);
    if constexpr (kFused) {  // the recheck's table: MaskS frame, one copy
        static_assert(kS2Waves * 64 >= 256, "one entry per thread");
        if (threadIdx.x < 256)
            reinterpret_cast<uint64_t *>(s_lds + kGearLdsBytes + kS2Waves * (kStageBytes + kQBytes))[threadIdx.x] =
                W.gear[threadIdx.x] << P.fs_sh;
    }
    __syncthreads();
    if (!kMaskL && threadIdx.x == 0) {
        dbg_ts(B, kTsScan + 4 * blockIdx.x + 1);
        if (blockIdx.x < 4096)
            dbg_ts(B, kTsHw + blockIdx.x,
                   uint64_t(__builtin_amdgcn_s_getreg(20 | (0 << 6) | (15 << 11))) << 32 |
                       uint32_t(__builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11))));
    }
    const char *tab = s_lds;
    if (!act) return;
    // Persistent mode (B.persist, k_scan / k_scan_f): one workgroup per CU;
    // every task comes from a per-launch atomic counter (W.tick[2], zeroed by
    // the host before the launch), so the CUs that run ahead take more of the
    // buffer, and a workgroup that starts late (its CU held by another
    // stream's kernel) finds the tasks taken instead of holding the launch.
    const bool persist = !kMaskL && B.persist != 0;
    auto next_task = [&]() { return wave_ticket(W.tick + 2); };
    for (uint32_t cur = persist ? next_task() : task;;) {
        if (cur >= B.total_tasks) break;
        scan_task<kMaskL, kFused>(B, P, W, s_lds, tab, cur, lane, wave, laneoff);
        if (!persist) break;
        cur = next_task();
    }
    if (clk && threadIdx.x == 0) {
        g_ts[clk + 2] = __builtin_amdgcn_s_memrealtime();
        g_ts[clk + 3] = __builtin_amdgcn_s_memtime();
    }
}

// One scan task: the 64 lane runs of task `task` (64 * B.scan_lane bytes of
// one buffer), staged through this wave's LDS slot.
template <bool kMaskL, bool kFused>
__device__ __forceinline__ void scan_task(const Batch &B, const DevParams &P, const Workspace &W, char *s_lds,
                                          const char *tab, uint32_t task, uint32_t lane, uint32_t wave,
                                          uint32_t laneoff)
{
    uint32_t b = 0;
    while (b + 1 < B.nbufs && task >= B.b[b + 1].task_base) ++b;
    const BufDesc &D = B.b[b];

    const uint64_t sl = B.scan_lane;                  // multiple of 128
    const uint64_t ub = reinterpret_cast<uint64_t>(D.data);
    const uint64_t lo_ok = ub & ~15ull, hi_ok = (ub + D.len + 15) & ~15ull;  // 16-B blocks of the buffer
    const uint64_t seg0 = uint64_t(task - D.task_base) * 64u;               // first lane run of the task
    if (seg0 * sl >= D.len) return;                                          // alignment padding task
    // this lane's run starts at s (buffer-relative); it tests [s, min(s + sl, len))
    const int64_t s = int64_t((seg0 + lane) * sl);
    // stage t of lane c covers [A(c) - 64 + kStage t, + kStage), A(c) = align16(ub + (seg0 + c) sl)
    // Staging starts kLead bytes before the run (>= W - 1 warm-up bytes); with
    // pair staging 128, so that its 128-B DMA chunks are whole HBM lines on a
    // 128-B aligned buffer (64-B aligned chunks straddle two lines: 40 % slower).
    constexpr uint32_t kLead = 128u;
    const uint32_t T = uint32_t((sl + kLead + (ub & 15u) + kStage - 1u) / kStage);
    const uint64_t wb = ((ub + seg0 * sl) & ~15ull) - kLead;  // lane 0's first stage
    const uint64_t base = wb > lo_ok ? wb : lo_ok;           // wave-uniform DMA base
    const uint64_t limw = hi_ok - 16u - base;                // last in-bounds piece (lane 0 is in bounds)
    const uint32_t lim = limw > 0x7FFFFFFFull ? 0x7FFFFFFFu : uint32_t(limw);
    const uint32_t ring = uint32_t(reinterpret_cast<uintptr_t>(s_lds)) + kGearLdsBytes + wave * kStageBytes;
    // Pair staging: DMA t carries 128 B (whole HBM lines) of each of the 32
    // runs of half t & 1 of the wave (4 instructions of 8 runs x 128 B), which
    // reads HBM ~14 % faster than 16 runs x 64 B (tools/ubench_mem.hip); half 1
    // runs one stage behind half 0.  Slot layout: run row r = lane & 31 at
    // 128 r, piece p at 16 (p ^ ((r >> 1) & 7)) (conflict-free ds_read_b128).
    // A register ping-pong instead of copies: even stages roll from A, odd
    // stages from Bv.  The half that loads at stage u (u & 1) reads its 128-B
    // row once, the first 64 B into stage u's array and the second 64 B into
    // the other array (stage u + 1's); the other half reads nothing.  The DMA
    // base advances in SGPRs (per-lane offsets fixed); only a wave whose
    // pieces could leave the buffer takes the clamped form.
    static_assert(kStage == 64 && kL == 4, "pair staging: 64-B stages, one slot");
    const uint32_t half = lane >> 5;
    const uint32_t row = lane & 31u, swz = (row >> 1) & 7u;
    // Half 1's runs are 32 runs after half 0's (lane lengths are multiples of
    // 256 B, so the 16-B alignment commutes): its pieces are half 0's offsets
    // plus the uniform 32 sl, added to the SGPR base.
    // offi[j] = piece j's offset - 1024 j (dma_stage_imm); for j >= 1 the run
    // is >= 8 runs (>= 4 KiB) past lane 0's, so the subtraction never wraps
    uint32_t offi[4];
    uint32_t om = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t r = 8u * j + lane / 8u;
        const uint32_t k = (lane % 8u) ^ ((r >> 1) & 7u);
        const uint32_t o = uint32_t((((ub + (seg0 + r) * sl) & ~15ull) - kLead + 16u * k) - base);  // wraps below base: clamped
        om = max(om, o);
        offi[j] = o - 1024u * j;
    }
    const uint64_t om0 = scan_wave_max(om);
    const uint64_t half_step = 32ull * sl;
    // kFast: the caller knows the pieces stay inside the buffer (the steady loop)
    auto issue = [&](auto PC, uint32_t u, auto FC) {
        constexpr uint32_t Q = decltype(PC)::value;  // u & 1: the half this DMA feeds
        constexpr bool kFast = decltype(FC)::value;
        const uint64_t adv = uint64_t(kStage) * (u - Q) + (Q ? half_step : 0ull);
#ifdef CDC_DIAG_NO_DMA
        return;  // build-time diagnostic only: no DMA (the slot keeps stale bytes), timing only
#endif
        if (kFast || om0 + adv <= uint64_t(lim)) {
#ifdef CDC_DIAG_L2
            // build-time diagnostic only: every DMA reads a 512-KiB window of
            // the buffer (L2-resident), wrong bytes, the scan's compute alone
            dma_stage_imm(lo_ok + ((base + adv - lo_ok) & 0x7FFF0ull), ring, offi);
#else
            dma_stage_imm(base + adv, ring, offi);
#endif
        } else {
            uint32_t eff[4];
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) eff[j] = min(offi[j] + 1024u * j + uint32_t(adv), lim);
            dma_stage(base, ring, eff);
        }
    };
    const char *rowp = s_lds + kGearLdsBytes + wave * kStageBytes + row * 128u;
    auto load_row = [&](uint4 (&first)[4], uint4 (&second)[4]) {
#ifdef CDC_DIAG_NO_ROW
        // build-time diagnostic only: no row reads (the registers keep stale bytes), timing only
        asm volatile("" : "+v"(first[0].x), "+v"(second[0].x));
        return;
#endif
#pragma unroll
        for (uint32_t g = 0; g < 4; ++g) first[g] = *reinterpret_cast<const uint4 *>(rowp + 16u * (g ^ swz));
#pragma unroll
        for (uint32_t g = 0; g < 4; ++g) second[g] = *reinterpret_cast<const uint4 *>(rowp + 16u * ((g + 4) ^ swz));
    };
    const uint32_t TT = T + 1;  // half 1 runs one stage behind
    const int32_t lag = int32_t(kStage * half);
    // the loop's key: the hi dword of the frame (k_scan_f: the bits MaskS and
    // MaskL share, in the frame fm_sh)
    const uint32_t vhi = to_vgpr(kFused ? P.fm_mi : kMaskL ? P.fl_hi : P.fs_hi);
    const uint32_t xlo = kMaskL ? P.fl_lo : P.fs_lo, xhi = kMaskL ? P.fl_hi : P.fs_hi;
    const int64_t rel0 = int64_t(((ub + uint64_t(s)) & ~15ull) - kLead) - int64_t(ub);
    using C0 = std::integral_constant<uint32_t, 0>;
    using C1 = std::integral_constant<uint32_t, 1>;
    using Gen = std::integral_constant<bool, false>;
    using Steady = std::integral_constant<bool, true>;

    uint4 A[4] = {}, Bv[4] = {};
#ifdef CDC_DIAG_WAITS
    // build-time diagnostic only: shader cycles this wave spends in the
    // per-stage DMA waits, its whole task and where it ran, to g_ts[kTsRes + 8 task]
    uint64_t wsum = 0;
    uint32_t nrc = 0;  // 32-byte groups whose filter fired in some lane (wave-uniform branch count)
    const uint64_t tk0 = __builtin_amdgcn_s_memtime();
    const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    // Stage 0 is not rolled: it lies 128 B (half 0) or 192 B (half 1) before
    // the run, and stage 1 alone gives fp >= 64 >= W - 1 warm-up bytes.  Its
    // loads and DMA issues are kept.
    static_assert(kLead >= 2 * kStage, "stage 0 must be pure warm-up for both halves");
    issue(C0{}, 0, Gen{});
    wait_vmcnt<0>();
    if (half == 0) load_row(A, Bv);  // stage 0 (unused) and stage 1 of half 0
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (1 < TT) issue(C1{}, 1, Gen{});
    if (1 < TT) {
        wait_vmcnt<0>();
        if (half == 1) load_row(Bv, A);  // stages 1 and 2 of half 1
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (2 < TT) issue(C0{}, 2, Gen{});
    }
    uint64_t gv[2][16];
#pragma unroll
    for (int k = 0; k < 16; ++k) gv[0][k] = lds_gear(tab, gear_addr(laneoff, word_of(Bv[0], k >> 2), k));
    uint64_t fp = 0;
    uint64_t rec = 0;
    uint64_t recL = 0;  // k_scan_f: the run's MaskL record
    const int32_t rr0 = int32_t(rel0 - s) - lag;
    // The recheck queue.  A lane whose filter fired in a 32-byte group queues
    // that group -- fp before it, its offset in the run and the lane: 12 bytes
    // of LDS (k_scan_f: the offset and lane only, 4 bytes) -- and the wave
    // rechecks the queue, one item per lane, at the end of the task or when
    // the queue is full.
    // The group's bytes are read again from memory then (aligned 16-byte
    // loads, clamped into the buffer; bytes outside the run only feed
    // positions the valid mask drops), so nothing of the group has to stay in
    // registers.  Rechecked in queue order, each run's hits reach its lane in
    // position order (the record keeps its first kRunCap ascending).
    uint64_t *const qf = reinterpret_cast<uint64_t *>(s_lds + kGearLdsBytes + kS2Waves * kStageBytes + wave * kQBytes);
    uint32_t *const qm = reinterpret_cast<uint32_t *>(qf + kQCap);
    static_assert(kQCap == 64, "one flush pass: item j in lane j");
    uint32_t qn = 0;  // queued items (wave-uniform)
    // The recheck's Gear entry for byte k of a 16-byte block: k_scan's own
    // table; k_scan_f's one-copy MaskS-frame table (entry b at 8 b, after the
    // queues) -- its loop's table is in another frame.
    const char *const ftab = s_lds + kGearLdsBytes + kS2Waves * (kStageBytes + kQBytes);
    auto rgear = [&](const uint4 &d, int k) -> uint64_t {
        if constexpr (kFused)
            return lds_gear(ftab, __builtin_amdgcn_ubfe(word_of(d, k >> 2), uint32_t(k & 3) * 8u, 8u) << 3);
        else
            return lds_gear(tab, gear_addr(laneoff, word_of(d, k >> 2), k));
    };
    auto flush = [&]() {
        {
            const bool v = lane < qn;
            const uint32_t meta = qm[v ? lane : 0u];
            const uint32_t owner = meta >> 24;
            const int32_t r0 = int32_t(meta & 0xFFFFFFu) - 256;
            const int64_t so = int64_t((seg0 + owner) * sl);  // the owner's run [so, so + ln)
            const int32_t ln = so < int64_t(D.len) ? int32_t(min(int64_t(sl), int64_t(D.len) - so)) : 0;
            const uint64_t a = ub + uint64_t(so + r0);  // 16-B aligned
            auto clamp16 = [&](uint64_t x) { return min(max(x, lo_ok), hi_ok - 16u); };
            const uint4 d0 = gload16(clamp16(a)), d1 = gload16(clamp16(a + 16u));
            uint64_t f = 0;
            if constexpr (kFused) {
                // the loop's frame lacks MaskS's top bits: the fingerprint
                // before the group is rolled again, in the MaskS frame, from
                // the 64 bytes before it (bits < W depend on the last W bytes
                // only; before the buffer's start, clamped bytes feed
                // positions no walker reads)
                uint4 dw[4];
#pragma unroll
                for (int h = 0; h < 4; ++h) dw[h] = gload16(clamp16(a - 64u + 16u * uint32_t(h)));
#pragma unroll
                for (int k = 0; k < 64; ++k) f = (f << 1) + rgear(dw[k >> 4], k & 15);
            } else {
                f = qf[v ? lane : 0u];
            }
            uint32_t miss = 0, missL = 0;
#pragma unroll
            for (int k = 0; k < 32; ++k) {
                f = (f << 1) + rgear(k < 16 ? d0 : d1, k & 15);
                miss |= min(key_of(f, xlo, xhi), 1u) << k;
                if constexpr (kFused) missL |= min(key_of(f, P.fm_llo, P.fm_lhi), 1u) << k;
            }
            const int32_t lo = r0 < 0 ? -r0 : 0, hi = ln - r0;  // valid positions [0, ln) of the run
            uint32_t vm = lo >= 32 ? 0u : (0xFFFFFFFFu << lo);
            vm &= hi >= 32 ? 0xFFFFFFFFu : (hi <= 0 ? 0u : (1u << hi) - 1u);
            const uint32_t hm = v ? ~miss & vm : 0u;
            const uint32_t hmL = kFused && v ? ~missL & vm : 0u;
            uint64_t todo = __ballot(hm != 0 || hmL != 0);  // false positives drop out here
            while (todo) {
                const int i = int(__builtin_ctzll(todo));
                todo &= todo - 1;
                const uint32_t o = uint32_t(__builtin_amdgcn_readlane(int(owner), i));
                const int32_t ri = __builtin_amdgcn_readlane(r0, i);
                uint32_t m = uint32_t(__builtin_amdgcn_readlane(int(hm), i));
                uint32_t mL = kFused ? uint32_t(__builtin_amdgcn_readlane(int(hmL), i)) : 0u;
                if (lane == o) {
                    for (; m; m &= m - 1) record_hit(rec, ri + int32_t(__builtin_ctz(m)));
                    if constexpr (kFused)
                        for (; mL; mL &= mL - 1) record_hit(recL, ri + int32_t(__builtin_ctz(mL)));
                }
            }
        }
        qn = 0;
    };
    // One stage t of parity Q: rolls cur (stage t's data); at its last group
    // the half loading stage t + 1 fills nxt (stage t + 1) and cur (t + 2),
    // and once those reads retired the slot takes DMA t + 2.  The filter is
    // reduced over 32-byte groups (two 16-byte groups): one wave-uniform
    // branch per 32 bytes into the queue.
    uint64_t f0 = 0;   // fp before the current 32-byte group
    uint32_t acc = 0xFFFFFFFFu;
    // SC (Steady): stage t + 2 exists and its DMA stays inside the buffer, so
    // the stage runs with no bounds tests (the loop over stage pairs below).
    auto stage = [&](auto PC, auto SC, uint32_t t, uint4 (&cur_d)[4], uint4 (&nxt_d)[4]) {
        constexpr uint32_t Q = decltype(PC)::value;
        constexpr bool kSteady = decltype(SC)::value;
#pragma unroll
        for (uint32_t gi = 0; gi < kGroups; ++gi) {
            if (gi + 1 == kGroups && (kSteady || t + 1 < TT)) {
#ifdef CDC_DIAG_WAITS
                const uint64_t w0 = __builtin_amdgcn_s_memtime();
                wait_vmcnt<0>();  // DMA t + 1 landed
                wsum += __builtin_amdgcn_s_memtime() - w0;
#else
                wait_vmcnt<0>();  // DMA t + 1 landed
#endif
                if (half != Q) load_row(nxt_d, cur_d);
                asm volatile("" ::: "memory");
            }
            const uint4 nx = gi + 1 < kGroups ? cur_d[gi + 1] : nxt_d[0];
            uint64_t (&cg)[16] = gv[gi & 1];
            uint64_t (&ng)[16] = gv[(gi + 1) & 1];
            if ((gi & 1) == 0) {
                f0 = fp;
                acc = 0xFFFFFFFFu;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                // byte by byte: the next group's address and gather between the
                // links of the fingerprint chain (a dependent v_lshl_add_u64
                // waits ~9 cycles, an independent one issues every ~5)
#pragma unroll
                for (int k = 4 * q; k < 4 * q + 4; k += 2) {
                    const uint32_t a0 = gear_addr(laneoff, word_of(nx, k >> 2), k);
                    fp = (fp << 1) + cg[k];
                    ng[k] = lds_gear(tab, a0);
                    const uint32_t k0 = uint32_t(fp >> 32) & vhi;
                    const uint32_t a1 = gear_addr(laneoff, word_of(nx, (k + 1) >> 2), k + 1);
                    fp = (fp << 1) + cg[k + 1];
                    ng[k + 1] = lds_gear(tab, a1);
                    acc = umin3(acc, k0, uint32_t(fp >> 32) & vhi);
                    __builtin_amdgcn_sched_barrier(0);
                }
                __builtin_amdgcn_sched_barrier(0);
                if (q == 1 && gi + 1 == kGroups && (kSteady || t + 2 < TT)) {
                    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");  // the row reads precede these 8 gathers
                    issue(PC, t + 2, SC);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            if (gi & 1) {
#ifndef CDC_DIAG_NO_RECHECK
                const uint64_t fm = __ballot(acc == 0);
#ifdef CDC_DIAG_WAITS
                nrc += fm ? 1u : 0u;
#endif
                if (fm) [[unlikely]] {  // queue the lanes' 32-byte groups
                    const uint32_t nq = uint32_t(__popcll(fm));
                    if (qn + nq > kQCap) flush();
                    if (acc == 0) {
                        const uint32_t idx =
                            qn + __builtin_amdgcn_mbcnt_hi(uint32_t(fm >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(fm), 0u));
                        const int32_t r0 = rr0 + int32_t(kStage * t + 16u * (gi - 1));
                        if constexpr (!kFused) qf[idx] = f0;  // k_scan_f rolls it again
                        qm[idx] = uint32_t(r0 + 256) | (lane << 24);
                    }
                    qn += nq;
                }
#else
                rec += acc == 0 ? 1u : 0u;  // build-time diagnostic only: no recheck
#endif
            }
        }
    };
    if (1 < TT) stage(C1{}, Gen{}, 1, Bv, A);
    // Steady pairs (t, t + 1): t + 3 < TT, and DMA t + 3 -- the farthest
    // of the pair's, adv = 64 (t + 2) + 32 sl -- inside the buffer.  The
    // stages after them (at most the last three, or all of a clamped wave's)
    // test their bounds.
    const int64_t room = int64_t(lim) - int64_t(om0) - int64_t(half_step);
    const int64_t tf = room >= 128 ? room / 64 - 1 : 0;
    const uint32_t t_steady = uint32_t(max<int64_t>(2, min<int64_t>(int64_t(TT) - 3, tf)));
    uint32_t t = 2;
    for (; t < t_steady; t += 2) {
        stage(C0{}, Steady{}, t, A, Bv);
        stage(C1{}, Steady{}, t + 1, Bv, A);
    }
    for (; t < TT; t += 2) {
        stage(C0{}, Gen{}, t, A, Bv);
        if (t + 1 < TT) stage(C1{}, Gen{}, t + 1, Bv, A);
    }
    if (qn) flush();
    if (s < int64_t(D.len)) (kMaskL ? W.runsL : W.runs)[64ull * D.task_base + seg0 + lane] = rec;
    if constexpr (kFused) {
        if (s < int64_t(D.len)) W.runsL[64ull * D.task_base + seg0 + lane] = recL;
        if (lane == 0) W.validL[task] = 1u;
    }
    if (!kMaskL && lane == 0) dbg_ts(B, kTsScan + 4 * blockIdx.x + 2 + (wave & 1));  // end of waves 0 / 1
#ifdef CDC_DIAG_WAITS
    // 8 slots per task: DMA-wait cycles, task cycles, start / end (100 MHz),
    // HW_ID, XCC_ID, filter-fired groups, wave index in the workgroup
    if (lane == 0 && 8 * task + 7 < 8 * 16384) {
        uint64_t *o = g_ts + kTsRes + 8 * task;
        o[0] = wsum;
        o[1] = __builtin_amdgcn_s_memtime() - tk0;
        o[2] = rt0;
        o[3] = __builtin_amdgcn_s_memrealtime();
        o[4] = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));
        o[5] = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (15 << 11));
        o[6] = nrc;
        o[7] = wave;
    }
#endif
}

// CDC_SCAN_LB (build-time A/B, with CDC_SCAN_WAVES=8): the launch bound the
// scan is compiled for; 768 keeps an 8-wave scan at <= 168 VGPRs (the
// 12-wave budget), leaving room on each SIMD for a k_resolve wave.
#ifndef CDC_SCAN_LB
#define CDC_SCAN_LB (kS2Waves * 64)
#endif
__global__ __launch_bounds__(CDC_SCAN_LB) void k_scan(const Batch B, const DevParams P, const Workspace W)
{
    scan_body<false>(B, P, W);
}

__global__ __launch_bounds__(kS2Waves * 64) void k_scan_l(const Batch B, const DevParams P, const Workspace W)
{
    scan_body<true>(B, P, W);
}

// Both indexes in one pass (launched instead of k_scan + k_scan_l while the
// adaptive hint says the MaskL index is needed): the loop filters on the bits
// MaskS and MaskL share, in a frame whose hi dword holds them (one v_and and
// half a v_min3 per byte, as k_scan); the recheck tests both masks exactly.
__global__ __launch_bounds__(CDC_SCAN_LB) void k_scan_f(const Batch B, const DevParams P, const Workspace W)
{
    scan_body<false, true>(B, P, W);
}

// The adaptive MaskL probe: the selection test of k_scan_l alone (one wave
// per scan task, no LDS, so it runs beside other kernels), raising the hint
// when some task would need the MaskL index.  The probing group itself builds
// no index (its walkers raw-scan); the hint makes the next groups build it.
constexpr uint32_t kProbeWaves = 4;

__global__ __launch_bounds__(kProbeWaves * 64) void k_maskl_probe(const Batch B, const DevParams P, const Workspace W)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t task = blockIdx.x * kProbeWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (task >= B.total_tasks) return;
    uint32_t b = 0;
    while (b + 1 < B.nbufs && task >= B.b[b + 1].task_base) ++b;
    const BufDesc &D = B.b[b];
    const uint64_t t = task - D.task_base;
    if (t * 64ull * B.scan_lane >= D.len) return;
    if (maskl_needed(B, P, W, D, t, lane) && lane == 0 && B.maskl_hint)
        __hip_atomic_store(B.maskl_hint, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// DPP helpers (in-row lane shifts, no LDS round trip; ds_bpermute-based
// shuffles cost ~100+ cycles each on the walk's critical path).
constexpr int kDppRowShr = 0x110;  // row_shr:n = 0x110 + n

template <int N>
__device__ __forceinline__ uint64_t dpp_shr64_zero(uint64_t v)  // lanes (j & 15) < N read 0
{
    const uint32_t lo = __builtin_amdgcn_update_dpp(0u, uint32_t(v), kDppRowShr + N, 0xF, 0xF, true);
    const uint32_t hi = __builtin_amdgcn_update_dpp(0u, uint32_t(v >> 32), kDppRowShr + N, 0xF, 0xF, true);
    return (uint64_t(hi) << 32) | lo;
}

template <int N>
__device__ __forceinline__ uint32_t dpp_shr32_keep(uint32_t v)  // lanes without a source keep v
{
    return __builtin_amdgcn_update_dpp(v, v, kDppRowShr + N, 0xF, 0xF, false);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l)
{
    const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(uint32_t(v), l));
    const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(uint32_t(v >> 32), l));
    return (uint64_t(hi) << 32) | lo;
}

// Wave-wide minimum of a u32, uniform result: in-row DPP min, then the 4 row minima.
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x)
{
    x = min(x, dpp_shr32_keep<1>(x));
    x = min(x, dpp_shr32_keep<2>(x));
    x = min(x, dpp_shr32_keep<4>(x));
    x = min(x, dpp_shr32_keep<8>(x));
    // readlane returns int: compare as unsigned (0xFFFFFFFF is the "none" sentinel)
    const uint32_t r0 = uint32_t(__builtin_amdgcn_readlane(x, 15));
    const uint32_t r1 = uint32_t(__builtin_amdgcn_readlane(x, 31));
    const uint32_t r2 = uint32_t(__builtin_amdgcn_readlane(x, 47));
    const uint32_t r3 = uint32_t(__builtin_amdgcn_readlane(x, 63));
    return min(min(r0, r1), min(r2, r3));
}

// Self-test of the wave primitives (one wave): out[0] = lanes whose DPP
// weighted prefix differs from the serial sum, out[1] = 1 if the DPP wave
// minimum differs from the serial minimum; out[2..5] = diagnostics.
__global__ __launch_bounds__(64) void k_selftest_wave(const uint64_t *in, uint32_t *out)
{
    __shared__ uint64_t s_in[64];
    __shared__ uint64_t s_v[64];
    const uint32_t j = threadIdx.x;
    uint64_t g = in[j];
    s_in[j] = g;
    uint64_t v = g;
    v += dpp_shr64_zero<1>(v) << 1;
    v += dpp_shr64_zero<2>(v) << 2;
    v += dpp_shr64_zero<4>(v) << 4;
    v += dpp_shr64_zero<8>(v) << 8;
    s_v[j] = v;  // in-row result
    {
        const uint64_t f15 = readlane64(v, 15);
        const uint64_t f31 = readlane64(v, 31) + (f15 << 16);
        const uint64_t f47 = readlane64(v, 47) + (f31 << 16);
        const uint32_t row = j >> 4;
        const uint64_t carry = row == 0 ? 0ull : row == 1 ? f15 : row == 2 ? f31 : f47;
        v += carry << ((j & 15u) + 1u);
    }
    __syncthreads();
    uint64_t ref = 0;
    for (uint32_t k = 0; k <= j; ++k) ref = (ref << 1) + s_in[k];
    uint64_t rowref = 0;
    for (uint32_t k = j & ~15u; k <= j; ++k) rowref = (rowref << 1) + s_in[k];
    const uint32_t bad = ref != v ? 1u : 0u;
    const uint32_t badrow = rowref != s_v[j] ? 1u : 0u;
    // values with the top bit set (the "none" sentinel included) must compare unsigned
    auto xv = [&](uint32_t k) { return k >= 40 ? 0xFFFFFFFFu : (uint32_t(s_in[k] >> 32) | 0x80000000u); };
    const uint32_t m = wave_min_u32(xv(j));
    uint32_t mref = 0xFFFFFFFFu;
    for (uint32_t k = 0; k < 64; ++k) mref = min(mref, xv(k));
    const uint32_t mnone = wave_min_u32(j == 63 ? 0x7FFFFFFFu : 0xFFFFFFFFu);
    const uint32_t ba = uint32_t(g), bbv = uint32_t(g >> 32), bc = uint32_t(g >> 16);
    const uint32_t b3bad = __builtin_amdgcn_bitop3_b32(ba, bbv, bc, 0xEA) != ((ba & bbv) | bc) ? 1u : 0u;
    const uint64_t bb = __ballot(bad | (b3bad << 1)), br = __ballot(badrow);
    if (j == 0) {
        out[0] = uint32_t(__popcll(bb));
        out[1] = (m != mref ? 1u : 0u) | (mnone != 0x7FFFFFFFu ? 2u : 0u);
        out[2] = uint32_t(__popcll(br));
        out[3] = uint32_t(br);
        out[4] = m;
        out[5] = mref;
    }
}

// ---------------------------------------------------------------------------
// Wave-cooperative next(p).
// ---------------------------------------------------------------------------
// The rare paths (raw scans, index runs beyond the first 64) are inlined: as
// calls they forced more VGPRs (values kept live in callee-saved registers
// across the call).

struct WalkCtx {
    uint64_t ub;       // absolute address of byte 0
    uint64_t len;
    uint32_t final_;
    const g_u64 *runs;     // this buffer's index records (run q at runs[q])
    uint64_t sl;           // run length (scan lane bytes)
    double inv_sl;
    const lds_char *tab;
    uint32_t laneoff;
    uint32_t lane;
    const uint64_t *gear;   // the 256-entry table in device memory
    const g_u64 *runsL;     // this buffer's MaskL index records (null: no MaskL index)
    const g_u32 *validL;    // per scan task of the buffer: runsL holds its 64 records
    uint32_t *flags;  // the launch's flags (the abort word: bounded waits)
};

// Run record q of the buffer.
__device__ __forceinline__ uint64_t ld_run(const g_u64 *runs, uint64_t q) { return runs[q]; }

// (A 32-copy table for long raw scans, filled on first use: C3 +2-4 %, C1 -4 %
// from the 80-KiB workgroups; not kept.)

// First position in [lo, hi) whose fingerprint (reset to 0 before fz) hits the
// mask, by a raw scan: lane j rolls its own kRawLaneBytes slice of a block
// after a 64-byte warm-up.  Positions are buffer-relative.  ESH selects the
// table layout (8: 32 copies, v_perm addresses, conflict-free gathers).
template <uint32_t ESH>
__device__ uint64_t raw_scan(const WalkCtx &C, const lds_char *tab, uint32_t laneoff, uint64_t lo, uint64_t hi,
                             uint64_t fz, uint32_t mlo, uint32_t mhi)
{
    const uint64_t H = C.ub + hi, FZ = C.ub + fz;
    uint64_t x = C.ub + lo;
    // lane slices of up to kRawLaneBytes: a short range (a dense index run) is
    // spread over every lane, so the serial roll per lane stays short
    const uint64_t lb = min<uint64_t>(kRawLaneBytes, max<uint64_t>(64, ((hi - lo + 63) / 64 + 15) & ~15ull));
    while (x < H) {
        const uint64_t A = x & ~15ull;
        const uint64_t bend = min(A + 64ull * lb, H);
        const uint64_t ts = max(x, A + uint64_t(C.lane) * lb);
        const uint64_t te = min(bend, A + uint64_t(C.lane + 1) * lb);
        uint64_t hit = kNoHit;
        if (ts < te) {
            const uint64_t hs = ts >= FZ + kWarm ? ts - kWarm : FZ;
            uint64_t fp = 0;
            for (uint64_t a = hs & ~15ull; a < te; a += 16) {
                const uint4 d = gload16(a);
                if (a >= FZ && a >= ts && a + 16 <= te) {
                    const uint64_t fp0 = fp;
                    if (roll16_test<ESH>(d, fp, tab, laneoff, mlo, mhi) == 0) {
                        uint64_t f = fp0;
                        hit = group_first_hit<ESH>(d, f, a, ts, te, FZ, tab, laneoff, mlo, mhi);
                        break;
                    }
                } else if (a >= FZ && a + 16 <= ts) {
                    roll16<ESH>(d, fp, tab, laneoff);
                } else {
                    hit = group_first_hit<ESH>(d, fp, a, ts, te, FZ, tab, laneoff, mlo, mhi);
                    if (hit != kNoHit) break;
                }
            }
        }
        const uint64_t m = __ballot(hit != kNoHit);
        if (m) return readlane64(hit, __ffsll((unsigned long long)m) - 1) - C.ub;
        x = bend;
    }
    return kNoHit;
}

__device__ __forceinline__ uint64_t raw_first_hit(const WalkCtx &C, uint64_t lo, uint64_t hi, uint64_t fz,
                                               uint32_t mlo, uint32_t mhi)
{
    return raw_scan<kWEntShift>(C, C.tab, C.laneoff, lo, hi, fz, mlo, mhi);
}

// Truncated window: positions fz + j, j < W - 1, fingerprint started at 0 at
// fz.  fp_j = sum_{k<=j} G[b_k] << (j-k): a weighted inclusive scan over lanes,
// in-row by DPP (shifts 1, 2, 4, 8), then the carried prefixes of rows 0-2.
// `byte` is data[fz + lane], preloaded by the caller (valid lanes only).
__device__ uint64_t trunc_first_hit(const WalkCtx &C, const DevParams &P, uint64_t fz,
                                    uint64_t norm_end, uint64_t lim, uint32_t byte)
{
    const uint32_t j = C.lane;
    const uint64_t pos = fz + j;
    const bool valid = (j + 1 < P.win) && pos < lim;
    uint64_t v = valid ? lds_gear(C.tab, (byte << kWEntShift) | C.laneoff) : 0ull;
    v += dpp_shr64_zero<1>(v) << 1;
    v += dpp_shr64_zero<2>(v) << 2;
    v += dpp_shr64_zero<4>(v) << 4;
    v += dpp_shr64_zero<8>(v) << 8;
    {
        const uint64_t f15 = readlane64(v, 15);
        const uint64_t f31 = readlane64(v, 31) + (f15 << 16);
        const uint64_t f47 = readlane64(v, 47) + (f31 << 16);
        const uint32_t row = j >> 4;
        const uint64_t carry = row == 0 ? 0ull : row == 1 ? f15 : row == 2 ? f31 : f47;
        v += carry << ((j & 15u) + 1u);
    }
    const bool small = pos < norm_end;
    const uint32_t mlo = small ? P.ms_lo : P.ml_lo, mhi = small ? P.ms_hi : P.ml_hi;
    const uint64_t m = __ballot(valid && key_of(v, mlo, mhi) == 0);
    return m ? fz + uint64_t(__ffsll((unsigned long long)m) - 1) : kNoHit;
}

// Index run holding position x.
__device__ __forceinline__ uint64_t run_of(const WalkCtx &C, uint64_t x)
{
    uint64_t q = uint64_t(double(x) * C.inv_sl);
    if (q * C.sl > x) --q;
    else if ((q + 1) * C.sl <= x) ++q;
    return q;
}

// First stored candidate of a run record (run start rs) in [a, b), or kNoHit.
// Stored entries are the run's smallest kRunCap, ascending: the smallest one
// >= a is the run's first candidate >= a even when the run is dense.
__device__ __forceinline__ uint64_t rec_first(uint64_t rec, uint64_t rs, uint64_t a, uint64_t b)
{
    const uint32_t n = min(rec_cnt(rec), kRunCap);
    uint64_t best = kNoHit;
#pragma unroll
    for (int i = int(kRunCap) - 1; i >= 0; --i) {
        const uint64_t pos = rs + rec_ent(rec, uint32_t(i));
        if (uint32_t(i) < n && pos >= a && pos < b) best = pos;
    }
    return best;
}

// Resolve a wave's 64 consecutive run records (run r0 + lane, valid lanes
// `in`): the first candidate in [a, b), rescanning dense runs whose stored
// entries do not answer.  *done = false when none of these runs holds one.
__device__ uint64_t recs_first(const WalkCtx &C, const DevParams &P, uint64_t r0, bool in, uint64_t rec, uint64_t a,
                               uint64_t b, uint64_t fz, bool &done, bool maskl = false)
{
    const uint64_t rs = (r0 + C.lane) * C.sl;
    const uint64_t cand = in ? rec_first(rec, rs, a, b) : kNoHit;
    uint64_t mc = __ballot(cand != kNoHit);
    uint64_t md = __ballot(in && cand == kNoHit && rec_cnt(rec) > kRunCap);
    done = true;
    while (mc | md) {
        const int lf = mc ? __ffsll((unsigned long long)mc) - 1 : 64;
        const int ld = md ? __ffsll((unsigned long long)md) - 1 : 64;
        if (lf < ld) return readlane64(cand, lf);
        const uint64_t rr = r0 + uint64_t(ld);
        const uint64_t lo = max(a, rr * C.sl), hi = min(b, (rr + 1) * C.sl);
        const uint64_t h = raw_first_hit(C, lo, hi, fz, maskl ? P.ml_lo : P.ms_lo, maskl ? P.ml_hi : P.ms_hi);
        if (h != kNoHit) return h;
        md &= ~(1ull << ld);
    }
    done = false;
    return kNoHit;
}

// First full-window MaskS candidate in [a, b) from the run index.
__device__ __forceinline__ uint64_t index_first_hit(const WalkCtx &C, const DevParams &P, uint64_t a, uint64_t b,
                                                 uint64_t fz)
{
    const uint64_t rl = run_of(C, b - 1);
    for (uint64_t r0 = run_of(C, a); r0 <= rl; r0 += 64) {
        const bool in = r0 + C.lane <= rl;
        const uint64_t rec = in ? ld_run(C.runs, r0 + C.lane) : 0ull;
        bool done;
        const uint64_t h = recs_first(C, P, r0, in, rec, a, b, fz, done);
        if (done) return h;
    }
    return kNoHit;
}

// First full-window MaskL candidate in [a, b) (a >= the chunk's p + Normal, so
// every window is full): from the MaskL index for the scan tasks k_scan_l
// built (64 records per round trip, dense runs rescanned), by a raw scan for
// the others.
__device__ __forceinline__ uint64_t maskl_first_hit(const WalkCtx &C, const DevParams &P, uint64_t a, uint64_t b,
                                                 uint64_t fz)
{
    if (!C.runsL) return raw_first_hit(C, a, b, fz, P.ml_lo, P.ml_hi);
    const uint64_t ra = run_of(C, a), rl = run_of(C, b - 1);
    for (uint64_t r0 = ra & ~63ull; r0 <= rl; r0 += 64) {
        const uint64_t lo = max(a, r0 * C.sl), hi = min(b, (r0 + 64) * C.sl);
        if (C.validL[r0 >> 6]) {
            const bool in = r0 + C.lane >= ra && r0 + C.lane <= rl;
            const uint64_t rec = in ? ld_run(C.runsL, r0 + C.lane) : 0ull;
            bool done;
            const uint64_t h = recs_first(C, P, r0, in, rec, lo, hi, fz, done, true);
            if (done) return h;
        } else {
            const uint64_t h = raw_first_hit(C, lo, hi, fz, P.ml_lo, P.ml_hi);
            if (h != kNoHit) return h;
        }
    }
    return kNoHit;
}

// The reference's (*Chunker).Next + (*FastCDC).Algorithm for the chunk that
// starts at p: returns the next chunk start, len at the end of a final
// stream, or kUndet when the bytes present do not decide the cut.
// Common case in ONE global round trip: every lane issues, together, its
// truncated-window byte, the candidate count of one index block and two
// entries of the first two blocks.
__device__ __forceinline__ uint64_t next_node(const WalkCtx &C, const DevParams &P, uint64_t p)
{
    const uint64_t E = C.len, r = E - p;
    if (r <= P.min_size) return C.final_ ? E : kUndet;
    uint64_t n, norm = P.normal_size, lim;
    bool clipped = false;
    if (C.final_) {
        if (r >= P.max_size) {
            n = P.max_size;
        } else {
            n = r;
            if (r <= P.normal_size) norm = r;
        }
        lim = p + n;
    } else {
        n = P.max_size;  // more stream follows: the reference peeks a full MaxSize window
        lim = p + n;
        if (lim > E) {
            lim = E;
            clipped = true;
        }
    }
    const uint64_t fz = p + P.min_size;
    const uint64_t norm_end = p + norm;
    const uint64_t full0 = fz + (P.win - 1);
    const uint64_t s_end = min(norm_end, lim);
    const bool has_s = full0 < s_end;
    const uint32_t j = C.lane;
    // ---- fused loads
    const uint64_t tpos = fz + j;
    const bool tvalid = (j + 1 < P.win) && tpos < lim;
    const uint64_t r0 = has_s ? run_of(C, full0) : 0;
    const uint64_t rl = has_s ? run_of(C, s_end - 1) : 0;
    const bool rin = has_s && r0 + j <= rl;
    uint32_t byte = 0;
    uint64_t rec = 0;
    if (tvalid) byte = as_space<const g_u8>(C.ub)[tpos];
    if (rin) rec = ld_run(C.runs, r0 + j);
    // ---- truncated window [fz, fz + W - 1)
    uint64_t h = trunc_first_hit(C, P, fz, norm_end, lim, byte);
    if (h != kNoHit) return h + P.cut_adj;
    // ---- full-window MaskS candidates in [full0, s_end)
    if (has_s) {
        bool done;
        h = recs_first(C, P, r0, rin, rec, full0, s_end, fz, done);
        if (done) return h + P.cut_adj;
        if (r0 + 64 <= rl) {
            h = index_first_hit(C, P, (r0 + 64) * C.sl, s_end, fz);
            if (h != kNoHit) return h + P.cut_adj;
        }
    }
    // ---- MaskL region [p + Normal, p + n): the MaskL index, or a raw scan
    const uint64_t l_lo = max(norm_end, full0);
    if (l_lo < lim) {
        h = maskl_first_hit(C, P, l_lo, lim, fz);
        if (h != kNoHit) return h + P.cut_adj;
    }
    return clipped ? kUndet : p + n;
}

// ---------------------------------------------------------------------------
// Successor graph of a resolution segment (k_resolve).
//
// On ordinary data next(v) is the first full-window MaskS candidate in
// [v + Min + W - 1, v + Normal), plus cut_adj, unless the truncated window
// [v + Min, v + Min + W - 1) hits first.  So nearly every chunk start a walk
// visits is a "listed" node v = c + cut_adj of a stored candidate c.  A
// walker wave lists the nodes of its segment (at most kGNodes, two per lane)
// and every lane computes the successors of its own nodes at once: the
// truncated window rolled lane-serially from 17 dwords, the full-window
// search over the segment's run records preloaded into LDS (one round trip,
// with a 1-bit-per-run "holds a candidate" map to skip empty runs).  A node
// whose successor needs more (a dense run whose stored entries do not answer,
// the MaskL region, a clipped or end-of-buffer window, records beyond the
// preload) is kGHard: there the walk takes the exact next_node().  The walk
// then reads each listed node's successor (position and list index) with
// readlane, a few cycles per chunk instead of a global round trip.
// ---------------------------------------------------------------------------
constexpr uint32_t kGNodes = 128;      // listed nodes per segment (two per lane)
constexpr uint32_t kGRecs = 512;       // run records preloaded per wave
constexpr uint64_t kGHard = ~1ull;     // successor not decided by the graph
constexpr uint32_t kGNone = 0xFFFFu;   // not a listed node

typedef __attribute__((address_space(3))) uint64_t lds_u64;
struct GraphLds {
    lds_u64 *rec;   // [kGRecs] runs ra .. ra + nr - 1
    lds_u64 *bits;  // [kGRecs / 64] bit i: run ra + i holds a candidate (dense included)
    lds_u64 *node;  // [kGNodes] listed nodes, ascending
};
constexpr uint32_t kGExtra = kGRecs / 64 + kGNodes;  // words of bits + node

__device__ __forceinline__ lds_u64 *lds_words(void *p)  // a generic pointer to LDS as an LDS pointer
{
    return as_space<lds_u64>(uint32_t(reinterpret_cast<uintptr_t>(p)));
}

__device__ __forceinline__ GraphLds graph_lds(void *rec, void *extra)
{
    GraphLds L;
    L.rec = lds_words(rec);
    L.bits = lds_words(extra);
    L.node = L.bits + kGRecs / 64;
    return L;
}

// The chunk window next_node() works on for a chunk starting at p (r > Min).
struct ChunkWin {
    uint64_t fz, norm_end, lim;
};

__device__ __forceinline__ ChunkWin chunk_win(const WalkCtx &C, const DevParams &P, uint64_t p)
{
    const uint64_t r = C.len - p;
    uint64_t norm = P.normal_size, lim;
    if (C.final_) {
        uint64_t n;
        if (r >= P.max_size) {
            n = P.max_size;
        } else {
            n = r;
            if (r <= P.normal_size) norm = r;
        }
        lim = p + n;
    } else {
        lim = min(p + P.max_size, C.len);
    }
    return ChunkWin{p + P.min_size, p + norm, lim};
}

// next_node(v) computed by ONE lane from the preloaded records, or kGHard.
// Identical to next_node() wherever it does not return kGHard.  Latency
// order: the truncated window's 17 dwords are requested first, the record
// search (LDS only) runs while they are in flight, then the window is rolled
// with the next 8 Gear gathers always in flight.
__device__ __forceinline__ uint64_t graph_succ(const WalkCtx &C, const DevParams &P, const GraphLds &L, uint64_t ra,
                                               uint32_t nr, uint64_t v)
{
    const uint64_t E = C.len;
    if (v >= E || E - v <= P.min_size) return kGHard;      // last chunk: next_node decides
    if (!C.final_ && v + P.max_size > E) return kGHard;    // clipped window (kUndet or a cut)
    const ChunkWin w = chunk_win(C, P, v);
    const uint64_t fz = w.fz, full0 = fz + (P.win - 1);
    if (w.norm_end < full0 || w.lim < full0) return kGHard;  // truncated window not all MaskS / in range
    const uint64_t a = C.ub + fz;
    const uint64_t a4 = a & ~3ull, last = (C.ub + E - 1) & ~3ull;  // full0 <= E: the used dwords are in bounds
    const uint32_t sh = uint32_t(a & 3u);
    uint32_t dw[17];
#pragma unroll
    for (int k = 0; k < 17; ++k) dw[k] = *as_space<const g_u32>(min<uint64_t>(a4 + 4u * uint64_t(k), last));
    // ---- full-window MaskS candidates in [full0, s_end) from the records (while the bytes load)
    uint64_t full = kNoHit;  // kGHard: undecided by the records
    const uint64_t s_end = min(w.norm_end, w.lim);
    if (full0 < s_end) {
        const uint64_t rl = run_of(C, s_end - 1);
        uint64_t r = run_of(C, full0);
        for (;;) {
            if (r > rl) break;  // no candidate
            uint64_t i = r - ra;
            if (i >= nr) {
                full = kGHard;
                break;
            }
            uint32_t wd = uint32_t(i >> 6);
            uint64_t bits = L.bits[wd] & (~0ull << (i & 63u));
            while (!bits) {
                ++wd;
                if (uint64_t(wd) * 64u >= nr) break;
                bits = L.bits[wd];
            }
            if (!bits) {
                if (ra + nr <= rl) full = kGHard;  // else: the preload covers the rest, no candidate
                break;
            }
            i = uint64_t(wd) * 64u + uint64_t(__builtin_ctzll(bits));
            r = ra + i;
            if (r > rl) break;
            const uint64_t rec = L.rec[i];
            const uint64_t cand = rec_first(rec, r * C.sl, full0, s_end);
            if (cand != kNoHit) {
                full = cand + P.cut_adj;
                break;
            }
            if (rec_cnt(rec) > kRunCap) {  // dense: the stored entries do not answer
                full = kGHard;
                break;
            }
            ++r;
        }
    }
    if (full == kNoHit) full = max(w.norm_end, full0) < w.lim ? kGHard : w.lim;  // MaskL region / forced cut
    // ---- truncated window [fz, full0): fingerprint from 0 at fz, MaskS at every position; it decides first
    const uint32_t wm1 = P.win - 1;  // positions tested (<= 63)
    uint64_t fp = 0;
    uint32_t first = 63;
    uint32_t wd2[16];  // bytes fz + 4 k .. fz + 4 k + 3
#pragma unroll
    for (int k = 0; k < 16; ++k) wd2[k] = __builtin_amdgcn_alignbyte(dw[k + 1], dw[k], sh);
    uint64_t gq[2][8];
#pragma unroll
    for (int t = 0; t < 8; ++t) gq[0][t] = lds_gear(C.tab, wgear_addr(C.laneoff, wd2[t >> 2], t & 3));
#pragma unroll
    for (int grp = 0; grp < 8; ++grp) {
        if (grp + 1 < 8) {  // the next 8 gathers in flight while this group rolls
#pragma unroll
            for (int t = 0; t < 8; ++t)
                gq[(grp + 1) & 1][t] = lds_gear(C.tab, wgear_addr(C.laneoff, wd2[2 * (grp + 1) + (t >> 2)], t & 3));
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const uint32_t j = uint32_t(8 * grp + t);
            if (j >= 63) break;
            fp = (fp << 1) + gq[grp & 1][t];
            const bool hit = key_of(fp, P.ms_lo, P.ms_hi) == 0 && j < wm1;
            first = min(first, hit ? j : 63u);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    return first < wm1 ? fz + first + P.cut_adj : full;
}

// The segment's listed nodes and their successors, held two per lane.
struct Graph {
    uint32_t n;       // listed nodes (> kGNodes: overflow, graph unused)
    uint64_t v[2];    // node lane (+ 64 s)
    uint64_t sp[2];   // its successor, or kGHard
    uint32_t si[2];   // the successor's list index, or kGNone
};

__device__ __forceinline__ uint32_t graph_find(const GraphLds &L, uint32_t n, uint64_t x)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (L.node[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo < n && L.node[lo] == x ? lo : kGNone;
}

// Lane r: the index of the r-th set bit of m (any value when r >= popcount(m)).
__device__ __forceinline__ uint32_t mask_rank_pos(uint64_t m, uint32_t r)
{
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t w = 32; w; w >>= 1) {
        const uint32_t c = uint32_t(__popcll(m & ((1ull << w) - 1)));
        if (r >= c) {
            r -= c;
            m >>= w;
            pos += w;
        }
    }
    return pos;
}

// Wave-uniform list index of node x, or kGNone.
__device__ __forceinline__ uint32_t graph_lookup(const Graph &G, uint32_t lane, uint64_t x)
{
    if (G.n > kGNodes) return kGNone;
    const uint64_t m0 = __ballot(lane < G.n && G.v[0] == x);
    if (m0) return uint32_t(__ffsll((unsigned long long)m0) - 1);
    const uint64_t m1 = __ballot(lane + 64u < G.n && G.v[1] == x);
    return m1 ? 64u + uint32_t(__ffsll((unsigned long long)m1) - 1) : kGNone;
}

// Build the graph of segment [S0, S1): list, preload, successors.
__device__ __forceinline__ void graph_build(const WalkCtx &C, const DevParams &P, GraphLds &L, Graph &G, uint64_t S0, uint64_t S1,
                            const Batch &B, uint32_t tslot)
{
    const bool tg = (B.debug & kDbgGraph) && C.lane == 0;
    const uint32_t lane = C.lane;
    const uint64_t adj = P.cut_adj;
    const uint64_t clo = S0 + 1 - adj, chi = S1 - adj;  // candidates c with c + adj in (S0, S1); S0 is node 0
    const uint64_t ra = run_of(C, S0 >= adj ? S0 - adj : 0);  // <= run_of(clo), <= rneed
    const uint64_t rneed = run_of(C, min(C.len, S1 + P.normal_size) - 1);
    const uint32_t nr = uint32_t(min<uint64_t>(rneed - ra + 1, kGRecs));
    uint64_t recs[kGRecs / 64];
#pragma unroll
    for (uint32_t k = 0; k < kGRecs / 64; ++k) {
        const uint32_t i = 64u * k + lane;
        recs[k] = 64u * k < nr && i < nr ? ld_run(C.runs, ra + i) : 0ull;
    }
    uint32_t n = 1;  // node 0: the segment start (the speculative chain's first node)
    if (lane == 0) L.node[0] = S0;
    const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
    for (uint32_t k = 0; k < kGRecs / 64; ++k) {
        if (64u * k >= nr) break;
        const uint32_t i = 64u * k + lane;
        const uint64_t rec = recs[k];
        if (i < nr) L.rec[i] = rec;
        const uint64_t nb = __ballot(i < nr && rec_cnt(rec) != 0);
        if (lane == 0) L.bits[k] = nb;
        // stored entries with c in [clo, chi): a contiguous range of the (ascending) entries
        const uint64_t rs = (ra + i) * C.sl;
        const uint32_t cnt = i < nr ? min(rec_cnt(rec), kRunCap) : 0u;
        uint32_t e0 = kRunCap, e1 = 0;  // listed entries [e0, e1)
#pragma unroll
        for (uint32_t e = 0; e < kRunCap; ++e) {
            const uint64_t c = rs + rec_ent(rec, e);
            if (e < cnt && c >= clo && c < chi) {
                e0 = min(e0, e);
                e1 = e + 1;
            }
        }
        const uint32_t kk = e1 > e0 ? e1 - e0 : 0u;
        const uint64_t b0 = __ballot(kk & 1u), b1 = __ballot(kk & 2u), b2 = __ballot(kk & 4u);
        const uint32_t pre = uint32_t(__popcll(b0 & below) + 2 * __popcll(b1 & below) + 4 * __popcll(b2 & below));
#pragma unroll
        for (uint32_t e = 0; e < kRunCap; ++e) {
            const uint32_t o = n + pre + (e - e0);
            if (e >= e0 && e < e1 && o < kGNodes) L.node[o] = rs + rec_ent(rec, e) + adj;
        }
        n += uint32_t(__popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2));
    }
    for (uint32_t k = (nr + 63) / 64; k < kGRecs / 64; ++k)
        if (lane == 0) L.bits[k] = 0;
    G.n = n;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own LDS writes, read back by other lanes
    if (tg) dbg_ts(B, tslot + 5);
    if (n > kGNodes) return;
#pragma unroll 1
    for (uint32_t s = 0; s < 2; ++s) {
        if (64u * s >= n) break;
        const uint32_t i = 64u * s + lane;
        uint64_t v = kGHard, sp = kGHard;
        uint32_t si = kGNone;
        if (i < n) {
            v = L.node[i];
            sp = graph_succ(C, P, L, ra, nr, v);
            if (sp != kGHard && sp >= S0 && sp < S1) si = graph_find(L, n, sp);
        }
        if (tg) dbg_ts(B, tslot + 6 + s);
        if (s == 0) {
            G.v[0] = v;
            G.sp[0] = sp;
            G.si[0] = si;
        } else {
            G.v[1] = v;
            G.sp[1] = sp;
            G.si[1] = si;
        }
    }
    if (n <= 64) {
        G.v[1] = kGHard;
        G.sp[1] = kGHard;
        G.si[1] = kGNone;
    }
}

__device__ __forceinline__ uint32_t buf_of_seg(const Batch &B, uint32_t g)
{
    uint32_t b = 0;
    while (b + 1 < B.nbufs && g >= B.b[b + 1].seg_base) ++b;
    return b;
}

__device__ __forceinline__ WalkCtx make_ctx(const Batch &B, const BufDesc &D, const Workspace &W,
                                            const char *tab)
{
    WalkCtx C;
    C.ub = reinterpret_cast<uint64_t>(D.data);
    C.len = D.len;
    C.final_ = B.final_;
    C.runs = as_space<const g_u64>(reinterpret_cast<uintptr_t>(W.runs + 64ull * D.task_base));
    C.sl = B.scan_lane;
    C.inv_sl = 1.0 / double(B.scan_lane);
    C.tab = as_lds(tab);
    C.lane = threadIdx.x & 63u;
    C.laneoff = (C.lane & (kWCopies - 1u)) << 3;
    C.gear = W.gear;
    C.runsL = B.maskl_index ? as_space<const g_u64>(reinterpret_cast<uintptr_t>(W.runsL + 64ull * D.task_base)) : nullptr;
    C.validL = B.maskl_index ? as_space<const g_u32>(reinterpret_cast<uintptr_t>(W.validL + D.task_base)) : nullptr;
    C.flags = W.flags;
    return C;
}

// ---------------------------------------------------------------------------
// k_resolve: the chain resolution of every buffer of a launch group in ONE
// launch, one wave per resolution segment [S0, S1) (B.seg bytes, the last one
// clipped to the buffer).
//
//   A. Speculative chain: the walk from S0 (a guess) to the first node >= S1
//      (through the segment's successor graph, next_node() where the graph
//      cannot answer).  Its nodes (w1_nodes) and exit X_q are published at
//      once (granule xg); this phase never waits.
//   B. Junction: the true chain enters segment q at X_{q-1} when segment q - 1
//      is on it.  The wave walks from X_{q-1} until it lands on a node of some
//      segment's speculative chain (its own, or a later one's, published in
//      phase A): it merged into segment conv >= q, so segments q+1 .. conv are
//      skipped and the next piece starts at X_conv, exactly the entry that
//      segment conv + 1 assumed.  Published as LOCAL (conv, cut count).
//   C. Decoupled look-back over the lower segments of the buffer for E, the
//      next segment on the true chain, and O, the cuts before it.  A LOCAL
//      with conv == its own index ("trivial") composes by addition; the first
//      non-trivial LOCAL met is waited on until it is INCLUSIVE.
//   D. If q is on the chain (E == q), its piece's cuts are written at O; then
//      the INCLUSIVE status (E_q, O_q) is published.  The buffer's last
//      segment writes the result row.
//
// Hand-offs are 8-byte granules (tag + data) written by ONE relaxed agent
// store (sc1) and polled with relaxed agent loads: no fences, no acquire
// polls (MI355X_MICROARCH.md, visibility).  A wave waits on lower segments,
// and on higher segments' phase-A publications only; workgroups take their
// segments in dispatch order (a ticket), so everything waited on is running
// or will be dispatched once some wave finishes: no deadlock whatever the
// grid size.  Node lists live in registers (node i of a list in lane i); a
// junction walk longer than 64 nodes (chains that never merge), and the debug
// mode, flag the buffer: its last segment waits for every INCLUSIVE status of
// the buffer and resolves it by the sequential walk.  Cut rows are stored
// write-through, so the sequential rewrite is the last word.  The granules
// are zeroed by the scan kernel of the same launch group.
// ---------------------------------------------------------------------------
constexpr uint32_t kMaxList = 64;                // nodes per register list
constexpr uint64_t kX55 = (1ull << 55) - 1;      // xg: X in bits 0-54 (all ones: kUndet), node count 55-61,
constexpr uint64_t kXNodes = 1ull << 62;         //     62: the node list is readable, 63: X is published
constexpr uint64_t kKindLocal = 1ull << 62, kKindIncl = 2ull << 62;
constexpr uint64_t kKindAbort = 3ull << 62;      // a wait of this segment (or below it) gave up: E = end, O = 0
constexpr uint32_t kConvEnd = 0x3FFFFFu;         // LOCAL: the chain ends in this piece (or before it)
constexpr uint32_t kSegEnd = 0xFFFFFFu;          // INCLUSIVE: no further segment on the chain

__device__ __forceinline__ uint64_t ld_rlx(const uint64_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void st_rlx(uint64_t *p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void drain_stores()
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Poll a granule (every lane the same word) until it is non-zero (0 if the wait gave up).
__device__ __forceinline__ uint64_t wait_granule(const uint64_t *p, uint32_t *flags, uint64_t what)
{
    SpinGuard sp;
    for (;;) {
        const uint64_t v = readlane64(ld_rlx(p), 0);
        if (v || !sp.ok(flags, kWaitPrev, what, 0)) return v;
        __builtin_amdgcn_s_sleep(kSpinSleep);
    }
}

__device__ __forceinline__ uint64_t x_dec(uint64_t g) { return (g & kX55) == kX55 ? kUndet : (g & kX55); }
__device__ __forceinline__ uint64_t x_enc(uint64_t x, uint32_t ns)
{
    return (1ull << 63) | (uint64_t(ns) << 55) | (x == kUndet || x >= kX55 ? kX55 : x);
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v)
{
#pragma unroll
    for (int o = 32; o; o >>= 1) v += uint64_t(__shfl_xor((unsigned long long)v, o));
    return v;
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src)
{
    return uint64_t(__shfl((unsigned long long)v, int(src)));
}

// A cut row, stored write-through (two 8-byte relaxed agent stores).
__device__ __forceinline__ void put_cut(cdc_cut *out, uint64_t off, uint64_t len)
{
    uint64_t *w = reinterpret_cast<uint64_t *>(out);
    st_rlx(w, off);
    st_rlx(w + 1, len & 0xFFFFFFFFull);
}

// E (the next segment on the chain, kSegEnd: none) and O (the cuts before it)
// after segments 0 .. q - 1 of a buffer whose granules start at sg.
//
// Segment r's status is a transition of the state E: when E == r (r is on the
// chain) E becomes conv_r + 1 and its cuts are added; otherwise nothing
// changes.  The look-back reads the statuses 64 at a time (eight windows per
// round trip), lane j holding segment lo + j, down to the window with the
// nearest INCLUSIVE status, and composes the transitions of each window: by
// a prefix sum when every one is trivial (conv_r == r: the chain entered at
// lo + j runs through the whole window), else by pointer jumping over the
// lanes (6 rounds of shuffles).  The windows above are kept as one composite
// F of the first kJ entries of the window above (a chain leaves a window at
// most kJ segments past its end); a longer jump takes the slow path, q - 1's
// own INCLUSIVE status.
// (k_resolve capped at 128 VGPRs, so that a resolve workgroup fits beside a
// scan workgroup, spilled 153 registers: 48 us alone instead of 25, and the
// warm pipelined C1 rate fell from 4.70k to 4.31k GiB/s.  Not kept.)
constexpr uint32_t kJ = 8;
constexpr uint32_t kLbWin = 8;  // windows per round trip

// Inclusive prefix sum within each 16-lane row (DPP, no LDS round trip).
__device__ __forceinline__ uint32_t row_incl_sum32(uint32_t x)
{
    x += __builtin_amdgcn_update_dpp(0u, x, kDppRowShr + 1, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0u, x, kDppRowShr + 2, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0u, x, kDppRowShr + 4, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0u, x, kDppRowShr + 8, 0xF, 0xF, true);
    return x;
}

__device__ __noinline__ void lookback(const uint64_t *sg, uint32_t q, uint32_t lane, uint32_t &E, uint64_t &O,
                                      uint32_t *flags, bool &ab)
{
    uint32_t Fe = q + lane;  // F, lane t < kJ: entering at hi + 1 + t leaves E = Fe with Fo cuts added
    uint64_t Fo = 0;
    bool slow = false;
    for (int64_t lo0 = int64_t(q) - 64;; lo0 -= 64 * int64_t(kLbWin)) {
        if (lo0 + 64 <= 0 && lo0 < int64_t(q) - 64) goto slow_path;  // below segment 0 (never, unless statuses are stale)
        uint64_t sw[kLbWin];
#pragma unroll
        for (uint32_t w = 0; w < kLbWin; ++w) {
            const int64_t p = lo0 - 64 * int64_t(w) + int64_t(lane);
            sw[w] = p >= 0 ? ld_rlx(sg + p) : 0ull;
        }
#pragma unroll
        for (uint32_t w = 0; w < kLbWin; ++w) {
            const int64_t lo = lo0 - 64 * int64_t(w);
            const int64_t p = lo + int64_t(lane);
            const bool valid = p >= 0;
            uint64_t s = sw[w];
            {
                SpinGuard sp;
                while (__ballot(valid && !s)) {
                    if (!sp.ok(flags, kWaitLook, q, uint64_t(lo0))) {
                        E = kSegEnd;  // gave up: the launch reports CDC_E_DEVICE
                        O = 0;
                        ab = true;
                        return;
                    }
                    __builtin_amdgcn_s_sleep(kSpinSleep);
                    if (valid && !s) s = ld_rlx(sg + p);
                }
            }
            const uint64_t im = __ballot(valid && (s >> 62) >= 2);
            const int istar = im ? 63 - int(__builtin_clzll(im)) : -1;  // nearest INCLUSIVE / ABORTED (segment 0 always is)
            const bool rel = valid && int(lane) > istar;
            const uint32_t code = uint32_t((s >> 40) & 0x3FFFFFu);
            const uint64_t cnt = rel ? (s & ((1ull << 40) - 1)) : 0ull;
            uint32_t ce;
            uint64_t co;
            if (!__ballot(rel && code != 0)) {
                // every transition trivial: entering at lane t runs to the window's end, then through
                // F's entry 0.  Counts per segment fit 32 bits; only the lanes below kJ (row 0) and
                // entries above the INCLUSIVE one (any row) are used, so row prefixes plus the row
                // totals give each lane's suffix.
                const uint32_t c32 = uint32_t(cnt);
                const uint32_t incl = row_incl_sum32(c32);
                const uint32_t r0 = uint32_t(__builtin_amdgcn_readlane(int(incl), 15));
                const uint32_t r1 = uint32_t(__builtin_amdgcn_readlane(int(incl), 31));
                const uint32_t r2 = uint32_t(__builtin_amdgcn_readlane(int(incl), 47));
                const uint32_t r3 = uint32_t(__builtin_amdgcn_readlane(int(incl), 63));
                const uint32_t row = lane >> 4;
                const uint32_t before = (row > 0 ? r0 : 0u) + (row > 1 ? r1 : 0u) + (row > 2 ? r2 : 0u);
                const uint64_t tot = uint64_t(r0) + r1 + r2 + r3;
                ce = uint32_t(__builtin_amdgcn_readfirstlane(int(Fe)));
                co = readlane64(Fo, 0) + tot - uint64_t(before + incl - c32);
            } else {
                uint32_t nx = 126;  // next lane on the chain (>= 64: leaves the window; 127: the chain ends)
                uint64_t add = cnt;
                if (rel) nx = code == kConvEnd ? 127u : uint32_t(min<uint64_t>(uint64_t(lane) + code + 1, 64 + kJ));
#pragma unroll
                for (int r = 0; r < 6; ++r) {
                    const uint32_t src = min(nx, 63u);
                    const uint32_t tn = uint32_t(__shfl(int(nx), int(src)));
                    const uint64_t ta = shfl64(add, src);
                    if (nx < 64) {
                        add += ta;
                        nx = tn;
                    }
                }
                const uint32_t ft = nx >= 64 && nx < 64 + kJ ? nx - 64 : 0u;
                const uint32_t fe = uint32_t(__shfl(int(Fe), int(ft)));
                const uint64_t fo = shfl64(Fo, ft);
                if (__ballot(rel && nx == 64 + kJ)) slow = true;  // a jump past what F tracks
                ce = nx == 127 ? kSegEnd : fe;
                co = add + (nx == 127 ? 0ull : fo);
            }
            if (istar >= 0) {
                const uint64_t si = readlane64(s, istar);
                if ((si >> 62) == 3) {  // aborted below: so is this segment
                    E = kSegEnd;
                    O = 0;
                    ab = true;
                    return;
                }
                const uint32_t ep = uint32_t((si >> 38) & 0xFFFFFFu);
                const uint64_t op = si & ((1ull << 38) - 1);
                if (ep == kSegEnd) {
                    E = kSegEnd;
                    O = op;
                    return;
                }
                const int64_t t = int64_t(ep) - lo;
                if (slow || t >= 64 + int64_t(kJ)) goto slow_path;
                if (t >= 64) {  // passes this window: enters F directly
                    E = uint32_t(__builtin_amdgcn_readlane(int(Fe), int(t - 64)));
                    O = op + readlane64(Fo, int(t - 64));
                } else {
                    E = uint32_t(__builtin_amdgcn_readlane(int(ce), int(t)));
                    O = op + readlane64(co, int(t));
                }
                return;
            }
            Fe = ce;
            Fo = co;
        }
    }
slow_path:  // q - 1's own INCLUSIVE status
    uint64_t sq;
    SpinGuard sp;
    while (((sq = readlane64(ld_rlx(sg + q - 1), 0)) >> 62) < 2) {
        if (!sp.ok(flags, kWaitLookSlow, q, 0)) {
            E = kSegEnd;
            O = 0;
            ab = true;
            return;
        }
        __builtin_amdgcn_s_sleep(kSpinSleep);
    }
    if ((sq >> 62) == 3) {
        E = kSegEnd;
        O = 0;
        ab = true;
        return;
    }
    E = uint32_t((sq >> 38) & 0xFFFFFFu);
    O = sq & ((1ull << 38) - 1);
}

// A result row's status, settled once: the scan kernel marks every row
// pending, the buffer's last segment turns pending into its status, and a
// wave whose wait gave up stores CDC_E_DEVICE into every row of the launch
// group (after or before the last segment: the row ends CDC_E_DEVICE).
__device__ __forceinline__ void settle_row(cdc_result *res, int64_t st)
{
    int64_t pend = kRowPending;
    __hip_atomic_compare_exchange_strong(&res->status, &pend, st, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __noinline__ void abort_rows(const Batch &B, uint32_t lane)
{
    for (uint32_t i = lane; i < B.nbufs; i += 64)
        __hip_atomic_store(&B.b[i].res->status, int64_t(CDC_E_DEVICE), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The sequential walk of a whole buffer (debug mode, lists that overflow):
// one wave walks next() from offset 0 and writes the cut list and the result row.
__device__ __forceinline__ void resolve_sequential(const WalkCtx &C, const DevParams &P, const BufDesc &D)
{
    uint64_t p = 0, idx = 0;
    while (p < C.len) {
        const uint64_t nx = next_node(C, P, p);
        if (nx == kUndet) break;
        if (C.lane == 0 && idx < D.cap) put_cut(D.out + idx, p, nx - p);
        ++idx;
        p = nx;
    }
    if (C.lane == 0) {
        st_rlx(&D.res->ncuts, idx <= D.cap ? idx : D.cap);
        st_rlx(&D.res->consumed, p);
        st_rlx(&D.res->needed, idx);
        settle_row(D.res, idx <= D.cap ? CDC_OK : CDC_E_NOSPACE);
    }
}

__device__ __forceinline__ void resolve_segment(const Batch &B, const DevParams &P, const Workspace &W, uint32_t g,
                                                const char *tab, GraphLds L)
{
    const uint32_t b = buf_of_seg(B, g);
    const BufDesc &D = B.b[b];
    WalkCtx C = make_ctx(B, D, W, tab);
    const uint32_t lane = C.lane, base = D.seg_base, q = g - base;
    const uint64_t seg = B.seg, S0 = uint64_t(q) * seg, segE = S0 + seg, S1 = min(segE, C.len);
    const bool l0 = lane == 0;
    if (l0) dbg_ts(B, kTsRes + 8 * g);
    Graph G;
    graph_build(C, P, L, G, S0, S1, B, kTsRes + 8 * g);
    if (l0) dbg_ts(B, kTsRes + 8 * g + 1);
    bool ovf = false;
    // debug mode 2: buffer 0's first segment never publishes its exit, so its
    // successor's wait for it gives up (the device-abort path)
    const bool withhold = (B.debug & kDbgForceAbort) && g == 0 && D.nseg > 1;
    // ---- A (phase 0) and B (phase 1).  While the walk stays on listed nodes
    // of a graph that fits one register (n <= 64: every 1-MiB segment of
    // random data), it is a scalar loop over node indices collecting a bit
    // mask; the node list is then built lane-parallel.  Anything else (a
    // kGHard node, an unlisted successor, another segment) goes through the
    // general loop: the graph where it answers, next_node() elsewhere.
    const bool g64 = G.n <= 64;
    bool aborted = false;  // a bounded wait of this wave gave up (or saw the launch's abort word)
    uint64_t sv = kUndet, jv = kUndet, cv = kUndet;  // lane i: node i of the speculative chain / junction / merged-into list
    uint32_t ns = 0, c2 = 0, cns = 0, k = 0, cur = q, conv = kConvEnd, exact = 0;
    uint64_t X = kUndet, cX = kUndet, ex = kUndet;  // ex: the node after the piece
    uint64_t pm = 0;                                 // graph nodes on the speculative chain (g64)
    for (uint32_t phase = 0; phase < 2; ++phase) {
        uint64_t x;
        bool rec = true;  // false: x is recorded already, step from it
        bool done = false;
        if (phase == 0) {
            x = S0;
            if (g64) {  // node 0 is S0
                uint32_t gi = 0;
                for (;;) {
                    pm |= 1ull << gi;
                    const uint32_t nxt = uint32_t(__builtin_amdgcn_readlane(int(G.si[0]), int(gi)));
                    // successors ascend, so a node seen again means records that
                    // are not this launch's: stop (the walk below decides)
                    if (nxt == kGNone || nxt >= 64u || ((pm >> nxt) & 1ull)) break;
                    gi = nxt;
                }
                ns = uint32_t(__popcll(pm));
                sv = shfl64(G.v[0], mask_rank_pos(pm, lane));
                if (lane >= ns) sv = kUndet;
                const uint64_t sz = readlane64(G.sp[0], int(gi));
                if (sz == kGHard) {
                    x = readlane64(G.v[0], int(gi));
                    rec = false;
                } else {
                    x = sz;
                }
            }
        } else {
            if (q == 0) {  // the true chain starts at 0 = S0: its piece is the speculative chain
                conv = 0;
                k = 0;
                cv = sv;
                cns = ns;
                cX = X;
                ex = X;
                break;
            }
            const uint64_t xp = wait_granule(W.xg + g - 1, W.flags, g);  // its load drained this wave's node-list stores
            drain_stores();
            if (l0 && !withhold) st_rlx(W.xg + g, x_enc(X, ns) | kXNodes);
            if (!xp) {  // gave up: no entry, no piece
                aborted = true;
                ex = kUndet;
                break;
            }
            x = x_dec(xp);
            cur = q;
            cv = sv;
            cns = ns;
            cX = X;
            if (g64 && x >= S0 && x < segE) {
                const uint32_t ia = graph_lookup(G, lane, x);
                if (ia != kGNone) {
                    uint64_t pj = 0;
                    uint32_t gi = ia;
                    bool merged = false;
                    for (;;) {
                        if ((pm >> gi) & 1ull) {
                            merged = true;
                            break;
                        }
                        pj |= 1ull << gi;
                        const uint32_t nxt = uint32_t(__builtin_amdgcn_readlane(int(G.si[0]), int(gi)));
                        if (nxt == kGNone || nxt >= 64u || ((pj >> nxt) & 1ull)) break;
                        gi = nxt;
                    }
                    c2 = uint32_t(__popcll(pj));
                    jv = shfl64(G.v[0], mask_rank_pos(pj, lane));
                    if (lane >= c2) jv = kUndet;
                    const uint64_t vg = readlane64(G.v[0], int(gi));
                    if (merged) {
                        const uint64_t m = __ballot(lane < ns && sv == vg);
                        k = uint32_t(__ffsll((unsigned long long)m) - 1);
                        conv = q;
                        ex = X;
                        done = true;
                    } else {
                        const uint64_t sz = readlane64(G.sp[0], int(gi));
                        if (sz == kGHard) {
                            x = vg;
                            rec = false;
                        } else {
                            x = sz;
                        }
                    }
                }
            }
        }
        uint32_t idx = kGNone;
        if (!done) {
            if (rec && x < segE) idx = graph_lookup(G, lane, x);
            for (;;) {
                if (rec) {
                    if (x == kUndet || x >= C.len || (phase == 0 && x >= segE)) {  // the chain ends / leaves
                        ex = x;
                        break;
                    }
                    if (phase == 1) {
                        const uint64_t r = x / seg;
                        if (r != cur) {  // entered a later segment: its published speculative chain
                            // (phase A never waits, so the wait ends)
                            uint64_t xr;
                            SpinGuard sp;
                            for (;;) {
                                xr = readlane64(ld_rlx(W.xg + base + r), 0);
                                if (xr & kXNodes) break;
                                if (!sp.ok(W.flags, kWaitJunction, g, base + r)) {
                                    aborted = true;
                                    break;
                                }
                                __builtin_amdgcn_s_sleep(kSpinSleep);
                            }
                            cur = uint32_t(r);
                            const bool pub = (xr & kXNodes) != 0;
                            cns = pub ? uint32_t((xr >> 55) & 0x7Fu) : 0u;
                            cX = pub ? x_dec(xr) : kUndet;
                            cv = lane < cns ? ld_rlx(W.w1_nodes + size_t(base + r) * kMaxList + lane) : kUndet;
                        }
                        const uint64_t m = __ballot(lane < cns && cv == x);
                        if (m) {  // merged into segment cur's speculative chain
                            k = uint32_t(__ffsll((unsigned long long)m) - 1);
                            conv = cur;
                            ex = cX;
                            break;
                        }
                    }
                    const uint32_t n = phase == 0 ? ns : c2;
                    if (n >= kMaxList) {  // chains that do not merge: the buffer is resolved sequentially
                        ovf = true;
                        ex = kUndet;
                        break;
                    }
                    if (phase == 0) {
                        if (lane == n) sv = x;
                        ++ns;
                        if (g64 && idx != kGNone) pm |= 1ull << idx;
                    } else {
                        if (lane == n) jv = x;
                        ++c2;
                    }
                }
                rec = true;
                uint64_t s = kGHard, nx;
                uint32_t ni = kGNone;
                if (idx != kGNone) {
                    const int l = int(idx & 63u);
                    s = readlane64(idx < 64u ? G.sp[0] : G.sp[1], l);
                    ni = uint32_t(__builtin_amdgcn_readlane(int(idx < 64u ? G.si[0] : G.si[1]), l));
                }
                if (s != kGHard) {
                    nx = s;
                } else {
                    nx = next_node(C, P, x);
                    ni = nx < segE ? graph_lookup(G, lane, nx) : kGNone;
                    ++exact;
                }
                x = nx;
                idx = nx < segE ? ni : kGNone;
            }
        }
        if (phase == 0) {
            X = ex;
            if (ovf) ns = 0;
            // X at once; the node list (read only by junctions that cross into this
            // segment) is flagged readable once a later load has drained its stores
            if (lane < ns) st_rlx(W.w1_nodes + size_t(g) * kMaxList + lane, sv);
            if (l0 && !withhold) {
                st_rlx(W.xg + g, x_enc(X, ns));
                dbg_ts(B, kTsRes + 8 * g + 2);
            }
            if (q == 0) {
                drain_stores();
                if (l0 && !withhold) st_rlx(W.xg + g, x_enc(X, ns) | kXNodes);
            }
        }
    }
    // the piece: nodes jv[0 .. c2) then cv[k .. cns) when merged (conv != kConvEnd); ex follows the last one
    const uint32_t nodes = c2 + (conv != kConvEnd ? cns - k : 0u);
    const uint64_t cuts = nodes - ((nodes > 0 && ex == kUndet) ? 1u : 0u);
    const uint64_t *sgb = W.sg + base;
    if (ovf && l0) __hip_atomic_store(W.flags + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t E = 0;
    uint64_t O = 0;
    if (q > 0 && !aborted) {
        if (l0) st_rlx(W.sg + g, kKindLocal | (uint64_t(conv == kConvEnd ? kConvEnd : conv - q) << 40) | cuts);
        lookback(sgb, q, lane, E, O, W.flags, aborted);
    }
    if (l0) dbg_ts(B, kTsRes + 8 * g + 3);
    const bool on = E == q && !aborted;
    const bool fb = B.force_fallback != 0;
    if (on && !fb && nodes > 0) {
        auto node_at = [&](uint32_t u) -> uint64_t {
            const uint64_t fj = shfl64(jv, min(u, 63u));
            const uint64_t fc = shfl64(cv, min(u >= c2 ? k + (u - c2) : 0u, 63u));
            return u >= nodes ? ex : (u < c2 ? fj : fc);
        };
        for (uint32_t t0 = 0; t0 < nodes; t0 += 64) {
            const uint32_t t = t0 + lane;
            const uint64_t v = node_at(t), s = node_at(t + 1);
            if (t < nodes) {
                if (s == kUndet) {
                    st_rlx(&D.res->consumed, v);  // the last chunk is not decided yet
                } else {
                    if (O + t < D.cap) put_cut(D.out + O + t, v, s - v);
                    if (s >= C.len) st_rlx(&D.res->consumed, C.len);
                }
            }
        }
        drain_stores();
    }
    const uint32_t Eq = on ? (conv == kConvEnd ? kSegEnd : conv + 1) : E;
    const uint64_t Oq = O + (on ? cuts : 0ull);
    if (aborted) {  // an ABORTED status (look-back passes it up) and CDC_E_DEVICE in every row
        if (l0) st_rlx(W.sg + g, kKindAbort);
        abort_rows(B, lane);
        return;
    }
    if (l0) {
        st_rlx(W.sg + g, kKindIncl | (uint64_t(Eq) << 38) | Oq);
        dbg_ts(B, kTsRes + 8 * g + 4);
        if (!(B.debug & kDbgGraph)) {
            dbg_ts(B, kTsRes + 8 * g + 5, G.n);
            dbg_ts(B, kTsRes + 8 * g + 6, exact);
            dbg_ts(B, kTsRes + 8 * g + 7, c2);
        }
    }
    if (q + 1 != D.nseg) return;
    // ---- the buffer's last segment: the result row, or the sequential fallback
    if (fb || __hip_atomic_load(W.flags + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        for (uint32_t p0 = 0; p0 < q; p0 += 64) {
            const uint32_t p = p0 + lane;
            SpinGuard sp;
            while (__ballot(p < q && (ld_rlx(sgb + min(p, q - 1)) >> 62) < 2)) {
                if (!sp.ok(W.flags, kWaitLast, g, p0)) {
                    aborted = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(kSpinSleep);
            }
            if (aborted || __ballot(p < q && (ld_rlx(sgb + min(p, q - 1)) >> 62) == 3)) {
                abort_rows(B, lane);
                return;
            }
        }
        if (__hip_atomic_load(W.flags + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || fb) {
            resolve_sequential(C, P, D);
            return;
        }
    }
    if (l0) {
        const bool ab = __hip_atomic_load(W.flags + kAbortWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
        st_rlx(&D.res->ncuts, Oq <= D.cap ? Oq : D.cap);
        st_rlx(&D.res->needed, Oq);
        settle_row(D.res, ab ? CDC_E_DEVICE : Oq <= D.cap ? CDC_OK : CDC_E_NOSPACE);
    }
}

// Empty buffers have no segment to write their result row.
__device__ __forceinline__ void write_empty_rows(const Batch &B, uint32_t lane)
{
    for (uint32_t i = lane; i < B.nbufs; i += 64) {
        if (B.b[i].nseg == 0) {
            B.b[i].res->ncuts = 0;
            B.b[i].res->consumed = 0;
            B.b[i].res->needed = 0;
            if (B.total_tasks) settle_row(B.b[i].res, CDC_OK);  // marked pending by the scan kernel
            else B.b[i].res->status = CDC_OK;                   // no scan kernel ran
        }
    }
}

// CDC_RESOLVE_WAVES_PER_EU (build-time A/B): cap k_resolve's registers (3:
// <= 168 VGPRs) so that one of its waves fits on a SIMD beside the scan's
// waves of the next pass.
#ifdef CDC_RESOLVE_WAVES_PER_EU
#define CDC_RESOLVE_ATTR __attribute__((amdgpu_waves_per_eu(CDC_RESOLVE_WAVES_PER_EU)))
#else
#define CDC_RESOLVE_ATTR
#endif
__global__ CDC_RESOLVE_ATTR __launch_bounds__(kWalkWavesPerWG * 64) void k_resolve(const Batch B, const DevParams P, const Workspace W)
{
    __builtin_amdgcn_s_setprio(3);  // latency-bound: issue ahead of a co-resident scan (next batch)
    __shared__ uint64_t s_tab[256 * kWCopies];
    __shared__ uint64_t s_grec[kWalkWavesPerWG][kGRecs];
    __shared__ uint64_t s_gx[kWalkWavesPerWG][kGExtra];
    __shared__ uint32_t s_ticket;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    if (threadIdx.x == 0) s_ticket = __hip_atomic_fetch_add(W.tick, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    fill_gear_lds<kWalkWavesPerWG * 64, kWCopies>(s_tab, W.gear);
    __syncthreads();
    if (blockIdx.x == 0 && wave == 0) write_empty_rows(B, lane);
    const uint32_t g = uint32_t(__builtin_amdgcn_readfirstlane(s_ticket)) * kWalkWavesPerWG + wave;
    if (g < B.total_segs)
        resolve_segment(B, P, W, g, reinterpret_cast<const char *>(s_tab), graph_lds(s_grec[wave], s_gx[wave]));
}

// ---------------------------------------------------------------------------
// k_stream_read: the HBM stream-read rate SURVEY.md 8(d) asks to report beside
// the roofline (measured, not the 8 TB/s spec).  Every lane reads 16-byte
// pieces, four in flight, grid-stride over the buffer, and folds them into
// one XOR per workgroup (written, so the loads are not dead).
// ---------------------------------------------------------------------------
constexpr uint32_t kStreamThreads = 256;

__global__ __launch_bounds__(kStreamThreads) void k_stream_read(const uint4 *p, uint64_t n16, uint32_t *sink)
{
    const uint64_t stride = uint64_t(gridDim.x) * kStreamThreads;
    uint64_t i = uint64_t(blockIdx.x) * kStreamThreads + threadIdx.x;
    uint32_t x = 0;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
        x ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
    }
    for (; i < n16; i += stride) {
        const uint4 a = p[i];
        x ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    for (int o = 32; o; o >>= 1) x ^= uint32_t(__shfl_xor(int(x), o));
    if ((threadIdx.x & 63u) == 0) atomicXor(sink + blockIdx.x, x);
}

// The same read in whole 8-KiB pieces per wave (8 nontemporal 16-byte loads
// per lane in flight), pieces handed out round-robin over the waves of the grid.
__global__ __launch_bounds__(kStreamThreads) void k_stream_read_nt(const uint4 *p, uint64_t n16, uint32_t *sink)
{
    const uint64_t waves = uint64_t(gridDim.x) * (kStreamThreads / 64);
    const uint64_t w = uint64_t(blockIdx.x) * (kStreamThreads / 64) + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t x = 0;
    const uint64_t pieces = n16 / 512;  // 512 x 16 B = 8 KiB per wave step
    for (uint64_t q = w; q < pieces; q += waves) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 *b = reinterpret_cast<const u32x4 *>(p + q * 512 + lane);
        u32x4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = __builtin_nontemporal_load(b + 64 * k);
#pragma unroll
        for (int k = 0; k < 8; ++k) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    for (uint64_t i = pieces * 512 + uint64_t(blockIdx.x) * kStreamThreads + threadIdx.x; i < n16;
         i += uint64_t(gridDim.x) * kStreamThreads) {
        const uint4 a = p[i];
        x ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    for (int o = 32; o; o >>= 1) x ^= uint32_t(__shfl_xor(int(x), o));
    if (lane == 0) atomicXor(sink + blockIdx.x, x);
}

// The scan's own way in: LDS-DMA (global_load_lds_dwordx4, four 1-KiB pieces
// per 4-KiB step), each wave streaming a contiguous stretch into a two-slot
// ring with one step in flight behind the one it issues; nothing reads the LDS.
constexpr uint32_t kStreamLdsWaves = 4;

__global__ __launch_bounds__(kStreamLdsWaves * 64) void k_stream_read_lds(const uint8_t *p, uint64_t len, uint32_t *sink)
{
    __shared__ __attribute__((aligned(16))) char lds[kStreamLdsWaves * 2 * 4096];
    const uint32_t lane = threadIdx.x & 63u, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nw = uint64_t(gridDim.x) * kStreamLdsWaves, w = uint64_t(blockIdx.x) * kStreamLdsWaves + wave;
    const uint64_t steps = len / 4096, per = (steps + nw - 1) / nw;
    const uint64_t s0 = w * per, s1 = min(steps, s0 + per);
    uint32_t off[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) off[j] = 1024u * j + 16u * lane;
    const uint32_t slot = uint32_t(reinterpret_cast<uintptr_t>(lds)) + wave * 8192u;
    for (uint64_t q = s0; q < s1; ++q) {
        dma_stage(reinterpret_cast<uint64_t>(p) + q * 4096, slot + uint32_t((q - s0) & 1) * 4096u, off);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) sink[blockIdx.x] = *reinterpret_cast<const uint32_t *>(lds);
}

int launch_stream_read(const void *d_buf, uint64_t len, int reps, double *best_us, double *median_us, void *stream)
{
    if (!best_us || !median_us) return CDC_E_INVALID;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const uint64_t n16 = len / 16;
    if (n16 == 0 || reps <= 0 || (reinterpret_cast<uintptr_t>(d_buf) & 15u)) return CDC_E_INVALID;
    int cus = 0, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return CDC_E_DEVICE;
    const uint32_t wgs = uint32_t(cus) * 8u;  // 8 workgroups of 4 waves per CU
    uint32_t *sink = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (hipMalloc(&sink, wgs * 4) != hipSuccess) return CDC_E_DEVICE;
    int rc = CDC_OK;
    std::vector<float> ms, ms2, ms3;  // per form
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess ||
        hipMemsetAsync(sink, 0, wgs * 4, st) != hipSuccess) {
        rc = CDC_E_DEVICE;
    } else {
        // the three forms interleaved, so they see the same clock
        for (int r = 0; r < reps && rc == CDC_OK; ++r) {
            for (int v = 0; v < 3 && rc == CDC_OK; ++v) {
                float t = 0.f;
                const bool rec0 = hipEventRecord(e0, st) == hipSuccess;
                if (v == 0)
                    hipLaunchKernelGGL(k_stream_read, dim3(wgs), dim3(kStreamThreads), 0, st,
                                       static_cast<const uint4 *>(d_buf), n16, sink);
                else if (v == 1)
                    hipLaunchKernelGGL(k_stream_read_nt, dim3(wgs), dim3(kStreamThreads), 0, st,
                                       static_cast<const uint4 *>(d_buf), n16, sink);
                else  // 4 workgroups per CU: 32 KiB of LDS each
                    hipLaunchKernelGGL(k_stream_read_lds, dim3(wgs / 2), dim3(kStreamLdsWaves * 64), 0, st,
                                       static_cast<const uint8_t *>(d_buf), len & ~uint64_t(4095), sink);
                const bool rec1 = hipEventRecord(e1, st) == hipSuccess;
                if (!rec0 || !rec1 || hipGetLastError() != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
                    hipEventElapsedTime(&t, e0, e1) != hipSuccess)
                    rc = CDC_E_DEVICE;
                else
                    (v == 0 ? ms : v == 1 ? ms2 : ms3).push_back(t);
            }
        }
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(sink);
    if (rc != CDC_OK) return rc;
    std::vector<float> *by[3] = {&ms, &ms2, &ms3};
    for (int v = 0; v < 3; ++v) {
        std::vector<float> &m = *by[v];
        std::sort(m.begin(), m.end());
        best_us[v] = 1e3 * double(m.front());
        median_us[v] = 1e3 * double(m[m.size() / 2]);
    }
    return CDC_OK;
}

// ---------------------------------------------------------------------------
// Host side: planning and launching.
// ---------------------------------------------------------------------------
static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

int make_plan(const uint64_t *lens, int nbufs, const DevParams &P, Plan *plan)
{
    uint64_t maxlen = 0;
    for (int i = 0; i < nbufs; ++i) maxlen = lens[i] > maxlen ? lens[i] : maxlen;
    // Resolution segments of 16 Min (1 MiB at the default sizes): one k_resolve
    // wave each.  A segment's successor graph (~32 listed nodes on random data)
    // is built in one pass of lane-parallel work; 2 MiB segments needed a second
    // pass in 44 % of the waves (C1 resolution 30 vs 36 us), 512 KiB segments
    // saved no graph time and doubled the look-back.
    uint64_t mult = 16;
    if (const char *env = getenv("CDC_SEG_MULT")) {
        const long v = atol(env);
        if (v >= 2 && v <= 1024) mult = uint64_t(v);
    }
    uint64_t seg = mult * P.min_size;
    const uint64_t need = (maxlen + kMaxSegs - 1) / kMaxSegs;
    if (seg < need) seg = need;
    seg = (seg + 15) & ~15ull;
    plan->seg = seg;
    // Scan lane length: one scan workgroup per CU (a workgroup holds 112 KiB of
    // LDS), for a grid of at most CUs - 7 workgroups; lane lengths are
    // multiples of 256 B (odd multiples of 128 B ran slower), so 1 GiB takes
    // 249 workgroups of 5,632-B lanes.  Against CUs - 8 (238 workgroups) that
    // is +2.8 % pipelined from a cold start and +1 % for the isolated scan
    // warm, but -1.3 % pipelined warm (fewer CUs left beside the scan for the
    // previous pass's resolution).
    uint64_t total = 0;
    for (int i = 0; i < nbufs; ++i) total += lens[i];
    static const uint64_t cus = [] {
        int n = 0, dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        return uint64_t(n);
    }();
    // Persistent scan (CDC_SCAN_TASKS_PER_WAVE = k > 0): one workgroup per CU
    // pulling tasks of 64 lane runs from a counter, about k tasks per wave, so
    // that the CUs that run ahead take the tail.  Measured slower than the
    // static grid at every k (2: -3 %, 3: -4 %, 6: -12 % on the driver's
    // command; shorter lanes add lead bytes and a pipeline fill per task), so
    // the default is the static grid (0).
    static const uint64_t env_tpw = [] {
        const char *e = getenv("CDC_SCAN_TASKS_PER_WAVE");
        const long v = e ? atol(e) : 0;
        return uint64_t(v >= 0 && v <= 64 ? v : 0);
    }();
    // the calling thread's override (the backup pipeline's scans share the
    // device with digest launches, cdc_backup.cpp)
    const uint64_t persist_tpw = t_scan_tpw >= 0 && t_scan_tpw <= 64 ? uint64_t(t_scan_tpw) : env_tpw;
    uint64_t wgs = persist_tpw ? cus : (cus > 16 ? cus - 7 : cus);
    if (const char *env = getenv("CDC_SCAN_WGS")) {
        const long v = atol(env);
        if (v >= 1 && v <= 65536) wgs = uint64_t(v);
    }
    const uint64_t tpw = persist_tpw ? persist_tpw : 1;
    plan->persist = persist_tpw ? 1u : 0u;
    plan->scan_wgs = uint32_t(wgs);
    uint64_t want = (total + wgs * kS2Waves * 64 * tpw - 1) / (wgs * kS2Waves * 64 * tpw);
    want = (want + kLaneQuant - 1) / kLaneQuant * kLaneQuant;
    if (want < 512) want = (512 + kLaneQuant - 1) / kLaneQuant * kLaneQuant;
    if (want > kScanLaneBytes) want = kScanLaneBytes / kLaneQuant * kLaneQuant;
    // buffers split into tasks independently: lengthen the lane until the
    // grid fits the target (a full 256-workgroup grid ran 7 % slower on C2)
    auto grid_of = [&](uint64_t ln) {
        uint64_t t = 0;
        for (int i = 0; i < nbufs; ++i) t += (lens[i] + 64 * ln - 1) / (64 * ln);
        return (t + kS2Waves - 1) / kS2Waves;
    };
    while (want + kLaneQuant <= kScanLaneBytes && grid_of(want) > wgs * tpw) want += kLaneQuant;
    uint32_t lane = uint32_t(want);
    if (const char *env = getenv("CDC_SCAN_LANE_BYTES")) {
        const long v = atol(env);
        if (v >= 256 && v <= long(kMaxScanLane) && v % kLaneQuant == 0) lane = uint32_t(v);
    }
    plan->scan_lane = lane;
    const uint64_t task_bytes = 64ull * lane;
    uint64_t segs = 0, tasks = 0;
    for (int i = 0; i < nbufs; ++i) {
        segs += (lens[i] + seg - 1) / seg;
        tasks += (lens[i] + task_bytes - 1) / task_bytes;
    }
    if (segs >= 0xFFFF0000ull || tasks >= 0xFFFF0000ull) return CDC_E_INVALID;
    plan->total_segs = uint32_t(segs);
    plan->total_tasks = uint32_t(tasks);
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off = align_up(off + bytes, 256);
        return o;
    };
    plan->off_runs = take(tasks * 64 * 8);
    plan->off_w1_nodes = take(segs * 64 * 8);
    plan->off_xg = take(segs * 8);
    plan->off_sg = take(segs * 8);
    plan->off_flags = take((kMaxBufsPerLaunch + 4) * 4);  // per buffer + the abort word
    // [0] segment ticket, [2] persistent scan task counter
    plan->off_tick = take(16 * 4);
    plan->off_runsL = take(tasks * 64 * 8);
    plan->off_validL = take(tasks * 4);
    plan->bytes = off;
    return CDC_OK;
}

// Optional live profiling: hipEvents recorded on the launch stream around the
// scan kernel and around the whole pipeline of each launch group.
struct ProfRec {
    hipEvent_t e0, e1, e2;  // before the scan, after the scan, after k_resolve
    uint64_t scan_bytes;
};
static std::mutex g_prof_mu;
static bool g_prof_on = false;
static std::vector<ProfRec> g_prof_live, g_prof_pool;

static bool prof_begin(ProfRec &r, uint64_t bytes)
{
    std::lock_guard<std::mutex> lk(g_prof_mu);
    if (!g_prof_on) return false;
    if (!g_prof_pool.empty()) {
        r = g_prof_pool.back();
        g_prof_pool.pop_back();
    } else if (hipEventCreate(&r.e0) != hipSuccess || hipEventCreate(&r.e1) != hipSuccess ||
               hipEventCreate(&r.e2) != hipSuccess) {
        return false;
    }
    r.scan_bytes = bytes;
    return true;
}

int launch_batch(const Batch &B, const DevParams &P, const Workspace &W, void *stream)
{
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (B.nbufs == 0) return CDC_OK;
    uint64_t bytes = 0;
    for (uint32_t i = 0; i < B.nbufs; ++i) bytes += B.b[i].len;
    ProfRec pr;
    const bool prof = prof_begin(pr, bytes);
    // With profiling on, the events ride on the kernels' own dispatch packets
    // (hipExtLaunchKernelGGL): no extra barrier packets, no bubbles.
    const uint32_t need_wgs = (B.total_tasks + kS2Waves - 1) / kS2Waves;
    const dim3 sgrid(B.persist && B.scan_wgs < need_wgs ? B.scan_wgs : need_wgs), sblock(kS2Waves * 64);
    const bool fused = B.maskl_index && B.maskl_fused;  // k_scan_f: both indexes in one pass
    if (B.persist && B.total_tasks > 0 && hipMemsetAsync(W.tick + 2, 0, 4, st) != hipSuccess) return CDC_E_DEVICE;
    if (B.total_tasks == 0) {  // every buffer is empty
        if (prof) {
            (void)hipEventRecord(pr.e0, st);
            (void)hipEventRecord(pr.e1, st);
        }
    } else if (prof) {
        if (fused)
            hipExtLaunchKernelGGL(k_scan_f, sgrid, sblock, 0, st, pr.e0, pr.e1, 0, B, P, W);
        else
            hipExtLaunchKernelGGL(k_scan, sgrid, sblock, 0, st, pr.e0, pr.e1, 0, B, P, W);
    } else if (fused) {
        hipLaunchKernelGGL(k_scan_f, sgrid, sblock, 0, st, B, P, W);
    } else {
        hipLaunchKernelGGL(k_scan, sgrid, sblock, 0, st, B, P, W);
    }
#ifdef CDC_DIAG_SCAN_ONLY
    // build-time diagnostic only (-DCDC_DIAG_SCAN_ONLY, never in the shipped
    // library): the scan alone, no resolution, cut lists not written
    if (prof) {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        (void)hipEventRecord(pr.e2, st);
        g_prof_live.push_back(pr);
    }
    return hipGetLastError() == hipSuccess ? CDC_OK : CDC_E_DEVICE;
#endif
    // MaskL index of the tasks near long MaskS-free stretches (most workgroups
    // exit after one look at the MaskS index on ordinary data)
    if (B.total_tasks > 0 && B.maskl_index && !fused)
        hipLaunchKernelGGL(k_scan_l, dim3(need_wgs), sblock, 0, st, B, P, W);  // not persistent (workgroup vote)
    else if (B.total_tasks > 0 && B.maskl_probe)
        hipLaunchKernelGGL(k_maskl_probe, dim3((B.total_tasks + kProbeWaves - 1) / kProbeWaves), dim3(kProbeWaves * 64),
                           0, st, B, P, W);
    const dim3 rgrid(B.total_segs > 0 ? (B.total_segs + kWalkWavesPerWG - 1) / kWalkWavesPerWG : 1u);
    if (prof)
        hipExtLaunchKernelGGL(k_resolve, rgrid, dim3(kWalkWavesPerWG * 64), 0, st, nullptr, pr.e2, 0, B, P, W);
    else
        hipLaunchKernelGGL(k_resolve, rgrid, dim3(kWalkWavesPerWG * 64), 0, st, B, P, W);
    if (prof) {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        g_prof_live.push_back(pr);
    }
    return hipGetLastError() == hipSuccess ? CDC_OK : CDC_E_DEVICE;
}

}  // namespace cdc

extern "C" int cdc_selftest_wave(uint32_t *result6)
{
    if (!result6) return CDC_E_INVALID;
    uint64_t h_in[64];
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto &v : h_in) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        v = x;
    }
    uint64_t *d_in = nullptr;
    uint32_t *d_out = nullptr;
    if (hipMalloc(&d_in, sizeof(h_in)) != hipSuccess) return CDC_E_DEVICE;
    if (hipMalloc(&d_out, 6 * 4) != hipSuccess) return CDC_E_DEVICE;
    int st = CDC_OK;
    if (hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice) != hipSuccess) st = CDC_E_DEVICE;
    if (st == CDC_OK) {
        hipLaunchKernelGGL(cdc::k_selftest_wave, dim3(1), dim3(64), 0, nullptr, d_in, d_out);
        if (hipMemcpy(result6, d_out, 6 * 4, hipMemcpyDeviceToHost) != hipSuccess) st = CDC_E_DEVICE;
    }
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return st;
}

extern "C" int cdc_debug_timestamps(uint64_t *out, uint64_t n)
{
    if (!out || n > cdc::kTsSlots) return CDC_E_INVALID;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(cdc::g_ts), n * 8) == hipSuccess ? CDC_OK : CDC_E_DEVICE;
}

extern "C" int cdc_profile_enable(int on)
{
    std::lock_guard<std::mutex> lk(cdc::g_prof_mu);
    cdc::g_prof_on = on != 0;
    return CDC_OK;
}

extern "C" int cdc_profile_collect(double *scan_ms, double *pipeline_ms, uint64_t *launches,
                                   uint64_t *scan_bytes)
{
    std::vector<cdc::ProfRec> recs;
    {
        std::lock_guard<std::mutex> lk(cdc::g_prof_mu);
        recs.swap(cdc::g_prof_live);
    }
    double s = 0, t = 0;
    uint64_t bytes = 0;
    int st = CDC_OK;
    for (auto &r : recs) {
        float a = 0, b = 0;
        if (hipEventSynchronize(r.e2) != hipSuccess || hipEventElapsedTime(&a, r.e0, r.e1) != hipSuccess ||
            hipEventElapsedTime(&b, r.e0, r.e2) != hipSuccess)
            st = CDC_E_DEVICE;
        s += a;
        t += b;
        bytes += r.scan_bytes;
    }
    {
        std::lock_guard<std::mutex> lk(cdc::g_prof_mu);
        for (auto &r : recs) cdc::g_prof_pool.push_back(r);
    }
    if (scan_ms) *scan_ms = s;
    if (pipeline_ms) *pipeline_ms = t;
    if (launches) *launches = recs.size();
    if (scan_bytes) *scan_bytes = bytes;
    return st;
}

