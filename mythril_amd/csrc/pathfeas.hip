// pathfeas.hip — host side of libpathfeas.so: the C ABI declared in include/pathfeas.h.
//
// Single translation unit: the kernels (pf_eval.hip, pf_keccak.hip) are included so the
// launches need no relocatable device code.  All entry points serialise on one mutex and
// re-select the device, because Mythril's query funnel calls in from a new worker thread
// per query (mythril/support/model.py:99-117).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pathfeas.h"
#include "pf_eval.hip"
#include "pf_keccak.hip"

namespace {

std::mutex g_mu;
thread_local std::string g_err_tls;
std::string g_err;
// host work done outside g_mu (pf_batch_create's program checks) reports into t_err, moved
// into g_err under the lock afterwards
thread_local bool t_defer_err = false;
thread_local std::string t_err;

// One entry per initialised device (pf_init's mask): its library stream, timing events for
// the Keccak launches and the launch geometry inputs.  Batches live on one device each and
// carry their own counters and events, so launches of different batches never share scratch.
struct Dev {
    int id = -1;            // the HIP device
    int key = -1;           // what the API calls it: the device id (pf_init) or a context id
                            // >= PF_CONTEXT_BASE (pf_init_contexts: several per device)
    hipStream_t stream = nullptr;
    hipStream_t up_stream = nullptr;  // batch uploads, issued outside g_mu (pf_batch_create)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int num_cus = 256;
    hipStream_t last_stream = nullptr;  // see switch_stream
    // device blocks of freed batches, reused by later batches that fit: a query's batch is
    // created and freed per call, and hipMalloc + hipFree (which synchronises the device)
    // per buffer were a millisecond of the single-query latency
    std::vector<std::pair<void*, size_t>> pool;
    // timing events of freed batches, reused (hipEventCreate / Destroy per batch were two
    // runtime calls each on the single-query path); under g_pool_mu
    std::vector<hipEvent_t> ev_free;
};
// ascending keys.  The entries are heap objects that stay put until pf_shutdown, so a Dev*
// taken by pf_batch_create (which runs without g_mu) survives a concurrent pf_init /
// pf_init_contexts growing and re-sorting the vector; the vector itself is read and changed
// under g_devs_mu (and changed only while g_mu is held too, so readers under g_mu need no more).
std::vector<std::unique_ptr<Dev>> g_devs;
std::mutex g_devs_mu;
int g_default = -1;       // index in g_devs of the default device (lowest id)
// search-kernel waves launched per CU (PF_WAVES_PER_CU overrides both).  Measured on config 3
// (1024 sets x 65,536 candidates, profiles/r01_wavesweep.md): with the longest-first set order
// the full sweep peaks at 512 (finer slices even out the sets' unequal costs in the last round
// of waves; 64 was 17 % slower).  The early-exit search is a work queue of (set, chunk) items
// taken by a chip-filling grid: 16 waves per CU (4 per SIMD, the narrow kernels' occupancy;
// PF_WAVES_PER_CU_EARLY), chunks of g_early_chunk_groups 64-candidate groups
// (PF_EARLY_CHUNK_GROUPS).
uint32_t g_waves_per_cu_full = 512;
uint32_t g_waves_per_cu_early = 16;
uint32_t g_early_chunk_groups = 8;
// Early-exit searches of 2 .. g_probe_max_sets sets that all carry a parent / hint model
// (candidate 0) start with a probe launch: one wave per set evaluates only candidates 0..63,
// then the queue search runs behind it on the stream from candidate 64 and skips every set the
// probe decided.  Without it every wave of the chip-filling grid claims its item before any
// witness exists, so the grid evaluates one group per wave at 4 waves/SIMD and the candidate-0
// waves finish at that contention.  Measured (tools/search_overhead_probe.py,
// profiles/r04o_search_overhead_probe.log, after the striped counters made a grid of skipping
// waves cheap): 4 planted sets 0.130 -> 0.110 ms, 16: 0.175 -> 0.128 ms; one set 0.064 ->
// 0.071 ms and sets without a candidate-0 witness (16 unplanted: 0.237 -> 0.321 ms) lose, hence
// the conditions.  (Round 4 before the striped counters: a single funnel query 0.686 -> 0.770 ms
// with the probe on for every batch.)  PF_PROBE_MAX_SETS sets the bound, 0 turns it off.
// A set without variables counts as parented (all its candidates are candidate 0), and the
// caller's PF_FLAG_NO_PROBE skips the probe when it knows a set's candidate 0 misses (check_sets:
// a host hint model that leaves a root false — the probe of a long program then only delays
// the search behind it; profiles/r06_probe_rule.md).
uint32_t g_probe_max_sets = 64;

int fail(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (t_defer_err)
        t_err = buf;
    else
        g_err = buf;
    return -1;
}

#define HIPCHK(x)                                                                       \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) return fail("%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), \
                                          __FILE__, __LINE__);                          \
    } while (0)

struct Batch {
    int device;
    void* d_mem = nullptr;  // one device block holding every array below
    size_t mem_cap = 0;
    size_t n_ins, n_const, n_vars, n_parents, n_sets;
    uint32_t max_vars;
    size_t n_narrow = 0;    // d_order[0, n_narrow): sets whose programs write only W registers
                            // < PF_NW_NARROW (8-register kernels, 3 waves/SIMD); the rest run
                            // the 16-register kernels in a second launch
    std::vector<pf_set_desc> h_descs;
    pf_set_desc* d_descs = nullptr;
    uint4* d_code = nullptr;
    uint32_t* d_consts = nullptr;
    uint4* d_schema = nullptr;
    uint32_t* d_parents = nullptr;
    uint32_t* d_found = nullptr;
    uint32_t* d_order = nullptr;    // set ids, most expensive first (search-kernel wave order)
    bool all_parented = false;      // every set carries a parent / hint model (candidate 0) or
                                    // has no variables
    uint32_t* d_scratch = nullptr;  // this batch's t0 (u64 [4]), queue heads and counter lines (pf_bytecode.h)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    ~Batch() {  // the device block goes back to its device's pool first (release_batch)
        if (d_mem) hipFree(d_mem);
        if (ev0) hipEventDestroy(ev0);
        if (ev1) hipEventDestroy(ev1);
    }
};

// Temporary device buffer freed on every return path (HIPCHK returns early).
struct DevBuf {
    void* p = nullptr;
    ~DevBuf() { hipFree(p); }
    template <typename T>
    T* as() { return static_cast<T*>(p); }
};

Dev* find_dev(int key) {
    for (auto& d : g_devs)
        if (d->key == key) return d.get();
    return nullptr;
}

constexpr size_t kPoolBlocks = 8;
// the device pools have their own lock: pf_batch_create takes and returns blocks without
// g_mu (a search holds g_mu until its results are back)
std::mutex g_pool_mu;

// a device block of at least `bytes` from the device's pool (smallest that fits and wastes
// at most 4x), else a new one
void* pool_acquire(Dev* D, size_t bytes, size_t* cap) {
    std::lock_guard<std::mutex> pk(g_pool_mu);
    size_t best = SIZE_MAX;
    for (size_t i = 0; i < D->pool.size(); ++i)
        if (D->pool[i].second >= bytes && D->pool[i].second <= 4 * bytes + (1u << 20) &&
            (best == SIZE_MAX || D->pool[i].second < D->pool[best].second))
            best = i;
    if (best != SIZE_MAX) {
        void* p = D->pool[best].first;
        *cap = D->pool[best].second;
        D->pool.erase(D->pool.begin() + best);
        return p;
    }
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    *cap = bytes;
    return p;
}

// free a batch: its block is kept for reuse (the oldest block is released when the pool is
// full).  Called with no launch of the batch in flight (pf_batch_free drains the device).
// a block back into its device's pool (the oldest block is released when the pool is full)
void pool_release(Dev* D, void* p, size_t cap) {
    std::lock_guard<std::mutex> pk(g_pool_mu);
    if (D->pool.size() >= kPoolBlocks) {
        hipFree(D->pool.front().first);
        D->pool.erase(D->pool.begin());
    }
    D->pool.emplace_back(p, cap);
}

void release_batch(Dev* D, Batch* B) {
    if (D && B->d_mem) {
        pool_release(D, B->d_mem, B->mem_cap);
        B->d_mem = nullptr;
    }
    if (D) {
        std::lock_guard<std::mutex> pk(g_pool_mu);
        for (hipEvent_t* e : {&B->ev0, &B->ev1}) {
            if (*e && D->ev_free.size() < 64) {
                D->ev_free.push_back(*e);
                *e = nullptr;
            }
        }
    }
    delete B;
}

// an event from the device's free list, else a new one
hipError_t event_acquire(Dev* D, hipEvent_t* e) {
    {
        std::lock_guard<std::mutex> pk(g_pool_mu);
        if (!D->ev_free.empty()) {
            *e = D->ev_free.back();
            D->ev_free.pop_back();
            return hipSuccess;
        }
    }
    return hipEventCreate(e);
}

// A launch on a caller's stream (the *_dev entry points) returns without waiting; before the
// device's next launch on a different stream reuses the Keccak events or a batch it reads,
// that stream is drained.
int switch_stream(Dev* D, hipStream_t st) {
    if (D->last_stream && D->last_stream != st) HIPCHK(hipStreamSynchronize(D->last_stream));
    D->last_stream = st;
    return 0;
}

// select (and make current) a device: the default one for device < 0
Dev* use_dev(int device) {
    if (g_devs.empty()) {
        fail("pf_init() has not been called");
        return nullptr;
    }
    Dev* D = device < 0 ? g_devs[g_default].get() : find_dev(device);
    if (!D) {
        fail("device %d was not initialised by pf_init", device);
        return nullptr;
    }
    hipError_t e = hipSetDevice(D->id);
    if (e != hipSuccess) {
        fail("hipSetDevice(%d): %s", D->id, hipGetErrorString(e));
        return nullptr;
    }
    return D;
}

Batch* as_batch(uint64_t h) { return reinterpret_cast<Batch*>(static_cast<uintptr_t>(h)); }

hipStream_t pick_stream(Dev* D, void* s) { return s ? reinterpret_cast<hipStream_t>(s) : D->stream; }

// launch geometry for the search kernel: enough waves to fill the CUs several times over,
// each wave walking >= 64 candidates of one set.
void geometry(int num_cus, uint32_t n_sets, uint32_t budget, uint32_t flags, uint32_t* per_wave,
              uint32_t* slices) {
    if (flags & PF_FLAG_EARLY_EXIT) {
        // work-queue items: chunks of g_early_chunk_groups groups, larger when the batch
        // would make more than 64 items per wave — every item costs a claim (an L2 atomic,
        // ~14 ns per head) even when its set is already decided, which dominated planted
        // batches of 65,536 sets (tools/full_pass.py: 136 ms per 1M sets at 8 groups)
        const uint64_t groups = (budget + 63u) / 64u;
        const uint64_t max_items = (uint64_t)num_cus * g_waves_per_cu_early * 64u;
        uint64_t cg = std::max<uint64_t>(g_early_chunk_groups, (n_sets * groups + max_items - 1) / max_items);
        // small batches (the funnel's single queries, fork pairs): chunks small enough that
        // every wave slot of the grid gets an item, so a set without a witness among its
        // candidates takes one chunk's time per wave, not g_early_chunk_groups groups'
        const uint64_t slots = (uint64_t)num_cus * g_waves_per_cu_early;
        const uint64_t fill = (n_sets * groups + slots - 1) / slots;
        if (fill < cg) cg = fill;
        cg = std::max<uint64_t>(1, std::min<uint64_t>(cg, groups));
        *per_wave = (uint32_t)(cg * 64u);
        *slices = std::max<uint32_t>(1u, (budget + *per_wave - 1) / *per_wave);
        return;
    }
    const uint64_t target_waves =
        (uint64_t)num_cus * ((flags & PF_FLAG_EARLY_EXIT) ? g_waves_per_cu_early : g_waves_per_cu_full);
    uint64_t groups = (budget + 63u) / 64u;  // 64-candidate groups per set
    uint64_t sl = (target_waves + n_sets - 1) / std::max<uint32_t>(n_sets, 1u);
    sl = std::max<uint64_t>(1, std::min<uint64_t>(sl, groups));
    uint64_t gpw = (groups + sl - 1) / sl;  // groups per wave
    *per_wave = (uint32_t)(gpw * 64u);
    *slices = (uint32_t)((budget + *per_wave - 1) / *per_wave);
    if (*slices == 0) *slices = 1;
}

// Enqueue one search over batch B on stream st (B's device must be current).
int check_enqueue(Batch* B, uint64_t gseed, uint32_t budget, uint32_t flags, uint32_t timeout_ms,
                  uint32_t* d_found, hipStream_t st) {
    Dev* D = find_dev(B->device);
    unsigned long long* d_counters = reinterpret_cast<unsigned long long*>(B->d_scratch);
    uint64_t* d_t0 = reinterpret_cast<uint64_t*>(B->d_scratch + 8);
#ifndef PF_FULL_QUEUE
#define PF_FULL_QUEUE 1
#endif
    // t0 and the profiling slots at the front, the work-queue heads of both launch parts from
    // PF_EARLY_QUEUE_OFF, the counter lines from PF_COUNTER_OFF: one fill for all
    {
        const uint32_t nz = PF_SCRATCH_BYTES / 4, nf = (uint32_t)std::max<size_t>(B->n_sets, 1);
        const uint32_t blocks = std::min<uint32_t>((nz + nf + 255u) / 256u, 1024u);
        hipLaunchKernelGGL(pf_reset_kernel, dim3(blocks), dim3(256), 0, st, B->d_scratch, nz, d_found, nf);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(B->ev0, st));
    const uint64_t deadline = timeout_ms ? (uint64_t)timeout_ms * 100000ull : 0ull;  // 100 MHz
    const bool early = flags & PF_FLAG_EARLY_EXIT;
    // phase 0: the probe (early exit, small batches: candidates 0..63 of every set, one wave
    // per set); phase 1: the search over the whole budget, whose waves skip decided sets
    const bool probe = early && budget > 64u && B->n_sets >= 2 && B->n_sets <= g_probe_max_sets &&
                       B->all_parented && !(flags & PF_FLAG_NO_PROBE);
    for (int phase = probe ? 0 : 1; phase < 2; ++phase) {
    const uint32_t pbudget = phase == 0 ? 64u : budget;
    // the 8-register sets first, then the 16-register ones (usually none)
    for (int part = 0; part < 2; ++part) {
        const size_t first = part ? B->n_narrow : 0;
        const size_t n = part ? B->n_sets - B->n_narrow : B->n_narrow;
        if (n == 0 || budget == 0) continue;
        uint32_t per_wave, slices;
        // phase 1 after a probe: candidates 64.. only (the probe evaluated 0..63)
        const uint32_t cbegin = (phase == 1 && probe) ? 64u : 0u;
        geometry(D->num_cus, (uint32_t)n, pbudget - cbegin, flags, &per_wave, &slices);
        const uint64_t items = (uint64_t)n * slices;
        if (items > 0xffffffffull) return fail("batch too large: %llu waves", (unsigned long long)items);
        // early exit: a chip-filling grid of persistent waves takes the items from the queue
        // heads (zeroed above); full sweep: one wave per item
        const uint64_t waves = early ? std::min<uint64_t>(items, (uint64_t)D->num_cus * g_waves_per_cu_early)
                             : PF_FULL_QUEUE ? std::min<uint64_t>(items, (uint64_t)D->num_cus * 16u)
                                             : items;
        // each (phase, part) launch has its own heads, all zeroed by the reset above
        uint32_t* d_queue =
            B->d_scratch + PF_EARLY_QUEUE_OFF / 4 + (phase * 2 + part) * PF_EARLY_QUEUES * PF_EARLY_QUEUE_STRIDE;
        const uint32_t blocks = (uint32_t)((waves + PF_SEARCH_WG_WAVES - 1) / PF_SEARCH_WG_WAVES);
        hipLaunchKernelGGL(part == 0 ? (early ? pf_check_early_kernel : pf_check_kernel)
                                     : (early ? pf_check_early_r16_kernel : pf_check_r16_kernel),
                           dim3(blocks), dim3(64 * PF_SEARCH_WG_WAVES), 0, st, B->d_descs, B->d_order + first,
                           (uint32_t)n, B->d_code, B->d_consts, B->d_schema, B->d_parents,
                           gseed, pbudget, per_wave, slices, flags, deadline, d_t0, d_found, d_counters,
                           d_queue, cbegin);
        HIPCHK(hipGetLastError());
    }
    }
    HIPCHK(hipEventRecord(B->ev1, st));
    return 0;
}

// Pinned host staging for the counter lines and verdicts a search reads back: a copy into
// pageable memory is staged and synchronous in the runtime (two of them were ~25 us of a
// single-query search's ~45 us outside the kernel); one buffer for the process (every entry
// point that reads results back holds g_mu), grown on demand, never shrunk, kept to process
// exit.  nullptr (pageable fallback) if the allocation fails.
uint8_t* pinned_staging(size_t bytes) {
    struct Pin {
        uint8_t* p = nullptr;
        size_t cap = 0;
    };
    static Pin t;
    if (bytes > t.cap) {
        if (t.p) (void)hipHostFree(t.p);
        t.p = nullptr;
        t.cap = 0;
        const size_t cap = std::max<size_t>((bytes + 65535) & ~size_t(65535), 65536);
        void* p = nullptr;
        if (hipHostMalloc(&p, cap, hipHostMallocPortable) != hipSuccess) return nullptr;
        t.p = static_cast<uint8_t*>(p);
        t.cap = cap;
    }
    return t.p;
}

// Pinned host staging for batch uploads (pf_batch_create), separate from pinned_staging and
// guarded by its own lock: an upload fills and copies it without holding g_mu.
std::mutex g_up_mu;
uint8_t* upload_staging(size_t bytes) {
    static uint8_t* p = nullptr;
    static size_t cap = 0;
    if (bytes > cap) {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t c = std::max<size_t>((bytes + (1u << 20) - 1) & ~size_t((1u << 20) - 1), 1u << 20);
        void* q = nullptr;
        if (hipHostMalloc(&q, c, hipHostMallocPortable) != hipSuccess) return nullptr;
        p = static_cast<uint8_t*>(q);
        cap = c;
    }
    return p;
}

// Wait for B's last search on stream st and read its counters.
// counters and kernel time of the last launch; with `found`, the verdicts too, copied before
// the one stream synchronisation (a second round trip was ~4 % of a single query's search)
int check_collect(Batch* B, hipStream_t st, pf_stats* stats, std::vector<uint32_t>* found = nullptr) {
    constexpr size_t cbytes = PF_COUNTER_STRIPES * 128;
    const size_t nf = std::max<size_t>(B->n_sets, 1);
    unsigned long long hs[PF_COUNTER_STRIPES * 16];
    uint8_t* pin = pinned_staging(cbytes + (found ? nf * 4 : 0));
    const uint32_t* d_counters = B->d_scratch + PF_COUNTER_OFF / 4;
    if (found) found->assign(nf, 0u);
    if (found && pin && B->d_found == d_counters + cbytes / 4) {
        // the batch block keeps found[] right after the counter lines: one copy (each copy is
        // a blit dispatch serialised behind the search)
        HIPCHK(hipMemcpyAsync(pin, d_counters, cbytes + nf * 4, hipMemcpyDeviceToHost, st));
    } else {
        HIPCHK(hipMemcpyAsync(pin ? static_cast<void*>(pin) : static_cast<void*>(hs), d_counters, cbytes,
                              hipMemcpyDeviceToHost, st));
        if (found)
            HIPCHK(hipMemcpyAsync(pin ? static_cast<void*>(pin + cbytes) : static_cast<void*>(found->data()),
                                  B->d_found, nf * 4, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(hipStreamSynchronize(st));
    if (pin) {
        memcpy(hs, pin, cbytes);
        if (found) memcpy(found->data(), pin + cbytes, nf * 4);
    }
    unsigned long long h[4] = {0, 0, 0, 0};
    for (int i = 0; i < PF_COUNTER_STRIPES; i++)
        for (int k = 0; k < 4; k++) h[k] += hs[i * 16 + k];
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, B->ev0, B->ev1));
    if (stats) {
        stats->evals_full = h[0];
        stats->cands_decided = h[1];
        stats->ops = h[2];
        stats->kernel_ms = ms;
        stats->n_sat = 0;
        stats->timed_out = h[3] ? 1u : 0u;
    }
    return 0;
}

// The device form of a validated batch (traffic / unit bits already set): three
// semantics-preserving peepholes rewrite the program the kernel runs, never the caller's
// arrays (the oracles evaluate the program as lowered).  Each set is rewritten in a scratch
// copy (descriptors may share or reorder code ranges) and appended to code_out; every pass is
// one forward walk with per-register state.  Shared by pf_batch_create and the host-only test
// export pf_device_program.
//  1. ASSERT: folded into the last writer of its B register when that is a compare or bool op
//     (PF_I_ASSERT) — the conjunction's value does not depend on where the and happens, and
//     with PF_FLAG_SHORTCIRCUIT an earlier check only exits sooner (round 2 folded it only
//     into the instruction right before it).
//  2. W_MOV: a zero-extending move (its source holds a value no wider than the move — values
//     are kept zero-extended, so the move copies it unchanged) is deleted and the readers of
//     its destination, up to that register's next write, read the source — provided the
//     source is not rewritten before the last of them.
//  3. W_CONST: deleted when its register is read, until its next write, only as the a / b
//     operand of W-reading instructions (not SPILL or MOV); those take the constant directly
//     (PF_I_KA / PF_I_KB, the constant index in the register field, traffic bit cleared) and
//     the kernel reads it with one scalar load.
//     A constant is folded only when it fits the W_CONST's width: the W_CONST masks its value
//     at write-back, a folded operand is read raw (ADVICE r4 — the lowering never packs a
//     wider one, but pf_batch_create trusts nothing the caller packed).
// consts (n_const x 8 u32, set-relative indices resolved through const_off) may be null: then
// every constant is taken to fit (pf_device_program's callers that pass none).
bool const_fits(const uint32_t* consts, size_t n_const, uint32_t idx, uint32_t w) {
    if (!consts) return true;
    if (idx >= n_const) return false;
    const uint32_t* c = consts + 8 * (size_t)idx;
    for (uint32_t j = 0; j < 8; j++) {
        const uint32_t lo = 32u * j;
        const uint32_t keep = w >= lo + 32u ? 0xffffffffu : (w > lo ? (1u << (w - lo)) - 1u : 0u);
        if (c[j] & ~keep) return false;
    }
    return true;
}

// Sets [s0, s1) of the batch: their device programs appended to code_out, each set's
// code_off rewritten to its offset in code_out.
void device_program_range(const uint32_t* code_fixed, std::vector<pf_set_desc>& descs_out, size_t s0, size_t s1,
                          std::vector<uint32_t>& code_out, const uint32_t* consts, size_t n_const) {
    std::vector<uint32_t> P;      // the set being rewritten
    std::vector<uint8_t> drop;
    struct Pending {              // pass 3: the W_CONST a register holds, and its readers
        int64_t at = -1;
        bool ok = true;
        std::vector<uint32_t> readers;
    };
    Pending pend[PF_NW + 1];
    for (size_t s = s0; s < s1; s++) {
        pf_set_desc& d = descs_out[s];
        const uint32_t n = d.n_ins;
        P.assign(code_fixed + 4 * (size_t)d.code_off, code_fixed + 4 * ((size_t)d.code_off + n));
        drop.assign(n, 0);
        auto tr_of = [&](uint32_t i) { return (P[4 * i] >> 18) & 7u; };
        // ---- 1. ASSERT -> PF_I_ASSERT on the last writer of its register
        {
            int64_t last_b[PF_NB];
            for (int r = 0; r < PF_NB; r++) last_b[r] = -1;
            for (uint32_t i = 0; i < n; i++) {
                const uint32_t op = P[4 * i] & 0xffu;
                if (op == PF_ASSERT) {
                    const int64_t k = last_b[(P[4 * i + 1] >> 8) & 31u];
                    if (k >= 0) {
                        const uint32_t unit = pf_op_unit(P[4 * (size_t)k] & 0xffu);
                        if ((unit == PF_U_CMP || unit == PF_U_BOOL) && !(P[4 * (size_t)k] & PF_I_ASSERT)) {
                            P[4 * (size_t)k] |= PF_I_ASSERT;
                            drop[i] = 1;
                        }
                    }
                } else if (PF_OP_WRITES_B(op)) {
                    last_b[P[4 * i + 1] & 31u] = i;
                }
            }
        }
#ifndef PF_NO_MOV_FUSE
        // ---- 2. zero-extending W_MOV -> its readers read the source
        {
            uint32_t wwidth[PF_NW + 1];  // width of the value each W register holds now
            for (int r = 0; r <= PF_NW; r++) wwidth[r] = 0xffffffffu;
            for (uint32_t i = 0; i < n; i++) {
                if (drop[i]) continue;
                const uint32_t op = P[4 * i] & 0xffu, tr = tr_of(i), dst = P[4 * i + 1] & 0xffu;
                const uint32_t w = (P[4 * i] >> 8) & 0x3ffu;
                if (op != PF_W_MOV) {
                    if ((tr & PF_TR_WW) && dst <= PF_NW) wwidth[dst] = w;
                    continue;
                }
                const uint32_t src = (P[4 * i + 1] >> 8) & 0xffu;
                bool ok = src <= PF_NW && dst <= PF_NW && wwidth[src] <= w;
                uint32_t last = i;
                if (ok) {
                    bool src_dead = false;
                    for (uint32_t j = i + 1; j < n; j++) {
                        if (drop[j]) continue;
                        const uint32_t jtr = tr_of(j), jw1 = P[4 * j + 1];
                        const bool reads = ((jtr & PF_TR_RA) && ((jw1 >> 8) & 0xffu) == dst) ||
                                           ((jtr & PF_TR_RB) && ((jw1 >> 16) & 0xffu) == dst);
                        if (reads) {
                            if (src_dead) { ok = false; break; }
                            last = j;
                        }
                        if ((jtr & PF_TR_WW) && (jw1 & 0xffu) == dst) break;
                        if ((jtr & PF_TR_WW) && (jw1 & 0xffu) == src) src_dead = true;
                        if ((P[4 * j] & 0xffu) == PF_END) break;
                    }
                }
                if (!ok) {
                    if (dst <= PF_NW) wwidth[dst] = w;
                    continue;
                }
                for (uint32_t t = i + 1; t <= last; t++) {
                    const uint32_t jtr = tr_of(t);
                    uint32_t& w1 = P[4 * t + 1];
                    if ((jtr & PF_TR_RA) && ((w1 >> 8) & 0xffu) == dst) w1 = (w1 & ~0xff00u) | (src << 8);
                    if ((jtr & PF_TR_RB) && ((w1 >> 16) & 0xffu) == dst) w1 = (w1 & ~0xff0000u) | (src << 16);
                }
                drop[i] = 1;  // dst keeps its old value, which nothing reads before its next write
            }
        }
#endif
#ifndef PF_NO_CONST_FUSE
        // ---- 3. W_CONST -> constant operands of its readers
        {
            auto settle = [&](uint32_t r) {
                Pending& q = pend[r];
                if (q.at >= 0 && q.ok && !q.readers.empty()) {
                    const uint32_t k = P[4 * (size_t)q.at + 2];
                    for (uint32_t t : q.readers) {
                        uint32_t& w0 = P[4 * t];
                        uint32_t& w1 = P[4 * t + 1];
                        const uint32_t jtr = (w0 >> 18) & 7u;
                        if ((jtr & PF_TR_RA) && ((w1 >> 8) & 0xffu) == r) {
                            w0 = (w0 & ~(PF_TR_RA << 18)) | PF_I_KA;
                            w1 = (w1 & ~0xff00u) | (k << 8);
                        }
                        if ((jtr & PF_TR_RB) && ((w1 >> 16) & 0xffu) == r) {
                            w0 = (w0 & ~(PF_TR_RB << 18)) | PF_I_KB;
                            w1 = (w1 & ~0xff0000u) | (k << 16);
                        }
                    }
                    drop[q.at] = 1;
                }
                q.at = -1;
                q.ok = true;
                q.readers.clear();
            };
            for (uint32_t i = 0; i < n; i++) {
                if (drop[i]) continue;
                const uint32_t op = P[4 * i] & 0xffu, tr = tr_of(i), w1 = P[4 * i + 1];
                const uint32_t ra = (w1 >> 8) & 0xffu, rb = (w1 >> 16) & 0xffu, rd = w1 & 0xffu;
                if (op == PF_END) break;
                // reads first (an instruction may read and rewrite the same register)
                for (int side = 0; side < 2; side++) {
                    const uint32_t r = side ? rb : ra;
                    if (!(tr & (side ? PF_TR_RB : PF_TR_RA)) || r > PF_NW || pend[r].at < 0) continue;
                    if (side && (tr & PF_TR_RA) && ra == r) continue;  // the same register twice
                    if (op == PF_W_SPILL || op == PF_W_MOV) pend[r].ok = false;
                    else pend[r].readers.push_back(i);
                }
                if ((tr & PF_TR_WW) && rd <= PF_NW) {
                    settle(rd);
                    if (op == PF_W_CONST && P[4 * i + 2] <= 0xffu &&
                        const_fits(consts, n_const, d.const_off + P[4 * i + 2], (P[4 * i] >> 8) & 0x3ffu))
                        pend[rd].at = i;
                }
            }
            for (uint32_t r = 0; r <= PF_NW; r++) settle(r);
        }
#endif
#ifndef PF_NO_LDS_SPILL
        // ---- 4. spill slots -> LDS entries 1..3 of EXP's window table (PF_SPILL_LDS)
        // A segment is a SPILL of slot k and the FILLs of k before its next SPILL.  One whose
        // range holds no W_EXP takes entry 2 or 3 when free (entry 1 too if no B_UMUL_NOOVF
        // runs in it): the value never touches scratch.  Entries are handed out in program
        // order; a segment without a FILL stays (a dead store costs nothing more).
        {
            struct Seg {
                uint32_t spill, last;
                std::vector<uint32_t> fills;
            };
            std::vector<Seg> segs;
            int64_t open[PF_MAX_SPILL];
            for (int k = 0; k < PF_MAX_SPILL; k++) open[k] = -1;
            std::vector<uint32_t> exp_at, umul_at;
            for (uint32_t i = 0; i < n; i++) {
                if (drop[i]) continue;
                const uint32_t op = P[4 * i] & 0xffu, k = P[4 * i + 2] & (PF_MAX_SPILL - 1u);
                if (op == PF_END) break;
                if (op == PF_W_EXP) exp_at.push_back(i);
                if (op == PF_B_UMUL_NOOVF) umul_at.push_back(i);
                if (op == PF_W_SPILL || op == PF_B_SPILL) {
                    open[k] = (int64_t)segs.size();
                    segs.push_back(Seg{i, i, {}});
                } else if ((op == PF_W_FILL || op == PF_B_FILL) && open[k] >= 0) {
                    Seg& g = segs[(size_t)open[k]];
                    g.fills.push_back(i);
                    g.last = i;
                }
            }
            auto any_in = [](const std::vector<uint32_t>& at, uint32_t lo, uint32_t hi) {
                const auto it = std::upper_bound(at.begin(), at.end(), lo);
                return it != at.end() && *it < hi;
            };
            int64_t busy_until[4] = {-1, -1, -1, -1};
            static const uint32_t order[3] = {2u, 3u, 1u};
            for (const Seg& g : segs) {
                if (g.fills.empty() || any_in(exp_at, g.spill, g.last)) continue;
                const bool umul = any_in(umul_at, g.spill, g.last);
                for (uint32_t e : order) {
                    if ((e == 1u && umul) || busy_until[e] >= (int64_t)g.spill) continue;
                    busy_until[e] = g.last;
                    P[4 * (size_t)g.spill + 2] = PF_SPILL_LDS | e;
                    for (uint32_t f : g.fills) P[4 * (size_t)f + 2] = PF_SPILL_LDS | e;
                    break;
                }
            }
        }
#endif
#ifndef PF_NO_FORWARD
        // ---- 5. back-to-back forwarding: an instruction reading the W register the kept
        // instruction right before it wrote takes that result directly (PF_I_FA / PF_I_FB,
        // traffic bit cleared), and the writer skips its write-back (PF_TR_WW cleared) when
        // no later instruction reads the register before its next write
        {
            int64_t prev = -1;
            for (uint32_t q = 0; q < n; q++) {
                if (drop[q]) continue;
                const int64_t p = prev;
                prev = q;
                uint32_t& qw0 = P[4 * q];
                const uint32_t qop = qw0 & 0xffu;
                if (qop == PF_END) break;
                if (p < 0) continue;
                uint32_t& pw0 = P[4 * (size_t)p];
                const uint32_t ptr = (pw0 >> 18) & 7u, pd = P[4 * (size_t)p + 1] & 0xffu;
                if (!(ptr & PF_TR_WW) || PF_OP_WRITES_B(pw0 & 0xffu) || pd > PF_NW) continue;
                const uint32_t qtr = (qw0 >> 18) & 7u, qw1 = P[4 * q + 1];
                const bool fa = (qtr & PF_TR_RA) && ((qw1 >> 8) & 0xffu) == pd;
                const bool fb = (qtr & PF_TR_RB) && ((qw1 >> 16) & 0xffu) == pd;
                if (!fa && !fb) continue;
                qw0 &= ~(((fa ? PF_TR_RA : 0u) | (fb ? PF_TR_RB : 0u)) << 18);
                qw0 |= (fa ? PF_I_FA : 0u) | (fb ? PF_I_FB : 0u);
                bool live = false;
                if (!((qtr & PF_TR_WW) && (qw1 & 0xffu) == pd)) {
                    for (uint32_t r = q + 1; r < n && !live; r++) {
                        if (drop[r]) continue;
                        const uint32_t rw0 = P[4 * r], rw1 = P[4 * r + 1], rtr = (rw0 >> 18) & 7u;
                        if ((rw0 & 0xffu) == PF_END) break;
                        live = ((rtr & PF_TR_RA) && ((rw1 >> 8) & 0xffu) == pd) ||
                               ((rtr & PF_TR_RB) && ((rw1 >> 16) & 0xffu) == pd);
                        if ((rtr & PF_TR_WW) && (rw1 & 0xffu) == pd) break;
                    }
                }
                if (!live) pw0 &= ~(PF_TR_WW << 18);
            }
        }
#endif
        const size_t first = code_out.size() / 4;
        size_t kept = 0;
        for (uint32_t i = 0; i < n; i++) kept += !drop[i];
        code_out.resize(4 * (first + kept));
        uint32_t* o = code_out.data() + 4 * first;
        for (uint32_t i = 0; i < n; i++)
            if (!drop[i]) {
                memcpy(o, P.data() + 4 * (size_t)i, 16);
                o += 4;
            }
        d.code_off = (uint32_t)first;
        d.n_ins = (uint32_t)kept;
    }
}

// Host threads for a batch's preparation and the set ranges they take (about equal
// instruction counts): one for small batches (a single query's), up to 8 for large ones.
std::vector<size_t> prep_ranges(const pf_set_desc* descs, size_t n_sets, size_t n_ins) {
    size_t nt = 1;
#ifndef PF_PREP_SERIAL
    if (n_sets >= 64 && n_ins >= (1u << 15)) {
        // hardware_concurrency reads sysfs: once per process, and not on a small batch's path
        static const size_t hw = std::max<size_t>(1, std::thread::hardware_concurrency());
        nt = std::min<size_t>({8, hw, n_sets / 32});
    }
#endif
    std::vector<size_t> cut(nt + 1, n_sets);
    cut[0] = 0;
    uint64_t total = 0, acc = 0;
    for (size_t s = 0; s < n_sets; s++) total += descs[s].n_ins;
    size_t t = 1;
    for (size_t s = 0; s < n_sets && t < nt; s++) {
        acc += descs[s].n_ins;
        if (acc * nt >= total * t) cut[t++] = s + 1;
    }
    return cut;
}

// fn(t) for t in [0, n) on the caller and n - 1 spawned threads
template <typename F>
void run_ranges(size_t n, F&& fn) {
    std::vector<std::thread> th;
    for (size_t t = 1; t < n; t++) th.emplace_back(fn, t);
    fn(0);
    for (auto& x : th) x.join();
}

// The device program of every set: each range of `cut` rewritten into its own buffer (on its
// own thread), then concatenated in set order — the program one pass over all sets gives.
void device_program(const uint32_t* code_fixed, size_t n_fixed, std::vector<pf_set_desc>& descs_out,
                    const std::vector<size_t>& cut, std::vector<uint32_t>& code_out, const uint32_t* consts,
                    size_t n_const) {
    const size_t nt = cut.size() - 1;
    code_out.clear();
    if (nt == 1) {
        code_out.reserve(n_fixed);
        device_program_range(code_fixed, descs_out, 0, descs_out.size(), code_out, consts, n_const);
        return;
    }
    std::vector<std::vector<uint32_t>> outs(nt);
    run_ranges(nt, [&](size_t t) {
        device_program_range(code_fixed, descs_out, cut[t], cut[t + 1], outs[t], consts, n_const);
    });
    size_t total = 0;
    for (const auto& o : outs) total += o.size();
    code_out.reserve(total);
    for (size_t t = 0; t < nt; t++) {
        const uint32_t base = (uint32_t)(code_out.size() / 4);
        for (size_t s = cut[t]; s < cut[t + 1]; s++) descs_out[s].code_off += base;
        code_out.insert(code_out.end(), outs[t].begin(), outs[t].end());
    }
}

}  // namespace

extern "C" {

int pf_version(void) { return 2; }

// Host only (no HIP call, tests/test_device_program.py): the program pf_batch_create would put
// on the device — traffic / unit bits recomputed from the opcodes, then the peepholes.
// code_out needs room for n_ins instructions (the peepholes only delete); descs_out n_sets.
int pf_device_program(const uint32_t* code, size_t n_ins, const uint32_t* consts, size_t n_const,
                      const pf_set_desc* descs, size_t n_sets, uint32_t* code_out, size_t* n_ins_out,
                      pf_set_desc* descs_out) {
    std::vector<uint32_t> fixed(code, code + 4 * n_ins);
    for (size_t i = 0; i < n_ins; i++) {
        uint32_t* I = fixed.data() + 4 * i;
        const uint32_t op = I[0] & 0xffu;
        I[0] = (I[0] & 0x3ffffu) | (pf_op_traffic(op) << 18) | (pf_op_unit(op) << 21);
    }
    std::vector<pf_set_desc> d(descs, descs + n_sets);
    std::vector<uint32_t> out;
    device_program(fixed.data(), fixed.size(), d, prep_ranges(descs, n_sets, n_ins), out, consts, n_const);
    memcpy(code_out, out.data(), out.size() * 4);
    *n_ins_out = out.size() / 4;
    memcpy(descs_out, d.data(), n_sets * sizeof(pf_set_desc));
    return 0;
}

#ifdef PF_PROFILE_UNITS
// profiling builds only (tools/unitprof.py): per-unit s_memtime cycles of a batch's last launch
int pf_prof_read(uint64_t handle, uint64_t* out) {
    std::lock_guard<std::mutex> lk(g_mu);
    Batch* B = as_batch(handle);
    if (!B || !use_dev(B->device)) return -1;
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(out, B->d_scratch + 2 * PF_PROF_SLOT, (PF_PROF_BUCKETS + 1) * 8,
                     hipMemcpyDeviceToHost));
    return 0;
}
#endif

const char* pf_last_error(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_err_tls = g_err;
    return g_err_tls.c_str();
}

int pf_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// The host lowering (libpflower.so) reports conflicts as C++ exceptions, and the first one
// thrown in a process has libgcc's unwinder set up its frame tables for every library then
// loaded — ~80 ms once the HIP runtime's are (tools/slow_job_probe.py: the corpus's first
// bucket whose hints meet a conflict took 80 ms, then 0.05 ms).  Both initialisers take that
// one-time cost here, with the runtime loaded, instead of the first query that conflicts.
void warm_unwinder() {
    static std::once_flag once;
    std::call_once(once, [] {
        try {
            throw std::runtime_error("unwinder warm-up");
        } catch (const std::exception&) {
        }
    });
}

// launch-geometry knobs from the environment, read by both initialisers
void read_env_knobs() {
    if (const char* e = getenv("PF_WAVES_PER_CU")) {
        long v = strtol(e, nullptr, 10);
        if (v >= 8 && v <= 4096) g_waves_per_cu_full = g_waves_per_cu_early = (uint32_t)v;
    }
    if (const char* e = getenv("PF_WAVES_PER_CU_EARLY")) {  // the early-exit search alone
        long v = strtol(e, nullptr, 10);
        if (v >= 1 && v <= 4096) g_waves_per_cu_early = (uint32_t)v;
    }
    if (const char* e = getenv("PF_PROBE_MAX_SETS")) {
        long v = strtol(e, nullptr, 10);
        if (v >= 0) g_probe_max_sets = (uint32_t)v;
    }
    if (const char* e = getenv("PF_EARLY_CHUNK_GROUPS")) {
        long v = strtol(e, nullptr, 10);
        if (v >= 1 && v <= 1024) g_early_chunk_groups = (uint32_t)v;
    }
}

// one more execution context (device id, API key) with its streams and events; called under
// g_mu, inserts under g_devs_mu keeping the keys ascending
int add_dev(int id, int key, const char* who) {
    HIPCHK(hipSetDevice(id));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, id));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail("%s: device %d is %s, this build targets gfx950", who, id, prop.gcnArchName);
    std::unique_ptr<Dev> D(new Dev());
    D->id = id;
    D->key = key;
    D->num_cus = prop.multiProcessorCount;
    HIPCHK(hipStreamCreateWithFlags(&D->stream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&D->up_stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreate(&D->ev0));
    HIPCHK(hipEventCreate(&D->ev1));
    std::lock_guard<std::mutex> dk(g_devs_mu);
    auto at = std::upper_bound(g_devs.begin(), g_devs.end(), key,
                               [](int k, const std::unique_ptr<Dev>& e) { return k < e->key; });
    g_devs.insert(at, std::move(D));
    g_default = 0;
    return 0;
}

int pf_init(uint64_t device_mask) {
    std::lock_guard<std::mutex> lk(g_mu);
    int n = 0;
    HIPCHK(hipGetDeviceCount(&n));
    if (device_mask == 0) return fail("pf_init: empty device mask");
    if (n < 64 && (device_mask >> n)) return fail("pf_init: mask %llx names devices beyond the %d visible",
                                                  (unsigned long long)device_mask, n);
    read_env_knobs();
    for (int id = 0; id < n && id < 64; ++id) {
        if (!((device_mask >> id) & 1ull) || find_dev(id)) continue;
        if (add_dev(id, id, "pf_init")) return -1;
    }
    warm_unwinder();
    return 0;
}

int pf_init_contexts(const int32_t* devices, size_t n, int32_t* ctx_out) {
    std::lock_guard<std::mutex> lk(g_mu);
    int nd = 0;
    HIPCHK(hipGetDeviceCount(&nd));
    if (!devices || !ctx_out || n == 0) return fail("pf_init_contexts: no devices");
    read_env_knobs();
    int next = PF_CONTEXT_BASE;
    for (const auto& D : g_devs) next = std::max(next, D->key + 1);
    for (size_t i = 0; i < n; ++i) {
        const int id = devices[i];
        if (id < 0 || id >= nd) return fail("pf_init_contexts: device %d of %d visible", id, nd);
        if (add_dev(id, next, "pf_init_contexts")) return -1;
        ctx_out[i] = next++;
    }
    warm_unwinder();
    return 0;
}

int pf_shutdown(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    std::lock_guard<std::mutex> dk(g_devs_mu);
    for (auto& D : g_devs) {
        hipSetDevice(D->id);
        hipDeviceSynchronize();
        {
            std::lock_guard<std::mutex> pk(g_pool_mu);
            for (auto& b : D->pool) hipFree(b.first);
            D->pool.clear();
            for (hipEvent_t e : D->ev_free) hipEventDestroy(e);
            D->ev_free.clear();
        }
        hipEventDestroy(D->ev0);
        hipEventDestroy(D->ev1);
        hipStreamDestroy(D->stream);
        if (D->up_stream) hipStreamDestroy(D->up_stream);
    }
    g_devs.clear();
    g_default = -1;
    return 0;
}

// Set s: its ranges, operands and schema checked against the batch, and its instructions
// copied into fixed[] (the set's own range) with the traffic / unit bits recomputed and
// register def-before-use checked; wide[s] set.  0 or fail().
static int check_set(size_t s, const uint32_t* code, size_t n_ins, size_t n_const, const uint32_t* schema,
                     size_t n_vars, size_t n_parents, const pf_set_desc* descs, uint32_t* fixed, uint8_t* wide) {
    {
        const pf_set_desc& d = descs[s];
        if ((uint64_t)d.code_off + d.n_ins > n_ins || d.n_ins == 0)
            return fail("set %zu: code range [%u,+%u) outside %zu instructions", s, d.code_off, d.n_ins, n_ins);
        if ((uint64_t)d.const_off + d.n_const > n_const)
            return fail("set %zu: constant range outside pool", s);
        if ((uint64_t)d.var_off + d.n_vars > n_vars) return fail("set %zu: schema range outside", s);
        if ((code[4 * ((size_t)d.code_off + d.n_ins - 1)] & 0xffu) != PF_END)
            return fail("set %zu: program does not end with PF_END", s);
        for (uint32_t i = 0; i < d.n_ins; i++) {
            const uint32_t* I = code + 4 * ((size_t)d.code_off + i);
            uint32_t op = I[0] & 0xffu, w = (I[0] >> 8) & 0x3ffu;
            if (op != PF_END && (w == 0 || w > PF_MAX_WIDTH))
                return fail("set %zu ins %u: width %u out of range", s, i, w);
            if ((op == PF_W_VAR || op == PF_B_VAR) && I[2] >= d.n_vars)
                return fail("set %zu ins %u: variable %u >= %u", s, i, I[2], d.n_vars);
            if (op == PF_W_CONST && I[2] >= d.n_const)
                return fail("set %zu ins %u: constant %u >= %u", s, i, I[2], d.n_const);
        }
        for (uint32_t v = 0; v < d.n_vars; v++) {
            const uint32_t* sc = schema + 4 * ((size_t)d.var_off + v);
            uint32_t kind = sc[0] & 0xffu, w = (sc[0] >> 8) & 0x3ffu;
            if (w == 0 || w > PF_MAX_WIDTH) return fail("set %zu var %u: width %u", s, v, w);
            if (sc[3] != PF_NO_PARENT && sc[3] >= n_parents) return fail("set %zu var %u: parent slot", s, v);
            if (kind == PF_VK_KECCAK && sc[1] >= d.n_const) return fail("set %zu var %u: keccak base", s, v);
            if (kind == PF_VK_ACTOR && (sc[2] > 4 || sc[1] + sc[2] > d.n_const))
                return fail("set %zu var %u: actor table", s, v);
            if (kind == PF_VK_CDBYTE && ((sc[1] & 0xffu) > 248u || (sc[1] & 7u) ||
                                         (sc[1] >> 20) + ((sc[1] >> 8) & 0xfffu) > d.n_const))
                return fail("set %zu var %u: calldata word constants", s, v);
        }
    }
    // traffic bits and register def-before-use, recomputed here so the kernel can trust
    // them whatever the caller packed (w0 bits 18..23)
    {
        const pf_set_desc& d = descs[s];
        memcpy(fixed + 4 * (size_t)d.code_off, code + 4 * (size_t)d.code_off, 16 * (size_t)d.n_ins);
        uint32_t wdef = 0u, bdef = 0u, max_wreg = 0u;
        uint64_t sdef = 0ull;
        for (uint32_t i = 0; i < d.n_ins; i++) {
            uint32_t* I = fixed + 4 * ((size_t)d.code_off + i);
            const uint32_t op = I[0] & 0xffu, tr = pf_op_traffic(op);
            I[0] = (I[0] & 0x3ffffu) | (tr << 18) | (pf_op_unit(op) << 21);
            const uint32_t rd = I[1] & 0xffu, ra = (I[1] >> 8) & 0xffu, rb = (I[1] >> 16) & 0xffu,
                           rc = (I[1] >> 24) & 0xffu;
            if ((tr & PF_TR_WW) && rd >= PF_NW) return fail("set %zu ins %u: W dst %u", s, i, rd);
            if (((tr & PF_TR_RA) && (ra >= PF_NW || !(wdef >> ra & 1u))) ||
                ((tr & PF_TR_RB) && (rb >= PF_NW || !(wdef >> rb & 1u))))
                return fail("set %zu ins %u: W register read before write", s, i);
            const bool bres = PF_OP_WRITES_B(op);
            const bool breads_ab = op >= PF_B_AND && op <= PF_B_XOR;
            if ((breads_ab && (!(bdef >> (ra & 31u) & 1u) || !(bdef >> (rb & 31u) & 1u))) ||
                ((op == PF_B_NOT || op == PF_ASSERT || op == PF_B_SPILL) && !(bdef >> (ra & 31u) & 1u)) ||
                ((op == PF_W_ITE || op == PF_B_ITE) && !(bdef >> (rc & 31u) & 1u)) ||
                (op == PF_B_ITE && (!(bdef >> (ra & 31u) & 1u) || !(bdef >> (rb & 31u) & 1u))))
                return fail("set %zu ins %u: B register read before write", s, i);
            if ((op == PF_W_SPILL || op == PF_W_FILL || op == PF_B_SPILL || op == PF_B_FILL) &&
                I[2] >= PF_MAX_SPILL)
                return fail("set %zu ins %u: spill slot %u >= %d", s, i, I[2], PF_MAX_SPILL);
            if (op == PF_W_SPILL || op == PF_B_SPILL) sdef |= 1ull << I[2];
            if ((op == PF_W_FILL || op == PF_B_FILL) && !(sdef >> I[2] & 1ull))
                return fail("set %zu ins %u: spill slot %u filled before it was spilled", s, i, I[2]);
            if (tr & PF_TR_WW) {
                wdef |= 1u << rd;
                max_wreg = std::max(max_wreg, rd);
            }
            if (i + 1 == d.n_ins) wide[s] = max_wreg >= PF_NW_NARROW;
            if (bres) bdef |= 1u << (rd & 31u);
        }
    }
    return 0;
}

// Host-side checks of packed programs and their device form (pf_batch_create and
// pf_eval_program): every kernel index is derived from these, so nothing the caller packed is
// trusted.  Fills the device program (device_program), the per-set wide flags and the largest
// variable count; returns 0 or fail().  A large batch (the corpus pass: 1,023 sets, 376k
// instructions, ~10 ms on one host thread) is checked and rewritten in set ranges on host
// threads, each range's device program appended to its own buffer, then concatenated in set
// order — the same program as the serial pass; a range that fails sends the whole batch
// through the serial pass, so the error reported is the first set's, as before.
static int prepare_program(const uint32_t* code, size_t n_ins, const uint32_t* consts, size_t n_const,
                           const uint32_t* schema, size_t n_vars, size_t n_parents, const pf_set_desc* descs,
                           size_t n_sets, std::vector<uint32_t>& code_out, std::vector<pf_set_desc>& descs_out,
                           std::vector<uint8_t>& wide, uint32_t& max_vars) {
    max_vars = 0;
    for (size_t s = 0; s < n_sets; s++) max_vars = std::max(max_vars, descs[s].n_vars);
    std::vector<uint32_t> code_fixed(4 * n_ins);
    wide.assign(n_sets, 0);
    descs_out.assign(descs, descs + n_sets);
    const std::vector<size_t> cut = prep_ranges(descs, n_sets, n_ins);
    const size_t nt = cut.size() - 1;
    bool bad = false;
    if (nt > 1) {
        std::vector<uint8_t> bad_t(nt, 0);
        const bool defer = t_defer_err;
        run_ranges(nt, [&](size_t t) {
            t_defer_err = true;  // a failing range's message stays on its thread: the serial pass reports
            for (size_t s = cut[t]; s < cut[t + 1] && !bad_t[t]; s++)
                bad_t[t] = check_set(s, code, n_ins, n_const, schema, n_vars, n_parents, descs, code_fixed.data(),
                                     wide.data()) != 0;
        });
        t_defer_err = defer;
        bad = std::find(bad_t.begin(), bad_t.end(), (uint8_t)1) != bad_t.end();
    }
    if (nt == 1 || bad) {
        for (size_t s = 0; s < n_sets; s++)
            if (check_set(s, code, n_ins, n_const, schema, n_vars, n_parents, descs, code_fixed.data(),
                          wide.data()))
                return -1;
    }
    device_program(code_fixed.data(), code_fixed.size(), descs_out, cut, code_out, consts, n_const);
    return 0;
}

int pf_batch_create_on(int device, const uint32_t* code, size_t n_ins, const uint32_t* consts,
                       size_t n_const, const uint32_t* schema, size_t n_vars,
                       const uint32_t* parents, size_t n_parents, const pf_set_desc* descs,
                       size_t n_sets, uint64_t* handle_out) {
    // The host half — checks, the device program, the wave order, the staging copy — touches
    // no library state and runs before the lock: a caller uploading the next batch from
    // another thread (tools/full_pass.py) overlaps it with a search in progress, which holds
    // the lock until its results are back.
    std::vector<uint32_t> code_out;
    std::vector<pf_set_desc> descs_out;
    std::vector<uint8_t> wide;
    uint32_t max_vars = 0;
    t_defer_err = true;
    const int prc = prepare_program(code, n_ins, consts, n_const, schema, n_vars, n_parents, descs, n_sets,
                                    code_out, descs_out, wide, max_vars);
    t_defer_err = false;
    if (prc) {
        std::lock_guard<std::mutex> lk(g_mu);
        g_err = t_err;
        return -1;
    }
    code = code_out.data();
    n_ins = code_out.size() / 4;
    descs = descs_out.data();
    // Longest-first wave order: waves are dispatched in index order, so mapping the first
    // waves to the most expensive sets leaves the cheap ones for the last, partly filled
    // round.  Weights are measured SIMD cycles per instruction relative to a cheap op
    // (EXP ~7.1k, a division ~2.6k, MUL ~750, cheap ~650).  8-register sets
    // come first (their launch precedes the 16-register one's).
    std::vector<uint64_t> cost(n_sets, 0);
    for (size_t s = 0; s < n_sets; ++s) {
        const uint4* I = reinterpret_cast<const uint4*>(code) + descs[s].code_off;
        uint64_t c = 0;
        for (uint32_t i = 0; i < descs[s].n_ins; ++i) {
            const uint32_t op = I[i].x & 0xffu;
            c += op == PF_W_EXP ? 110u : op == PF_W_MUL ? 12u : pf_op_unit(op) == PF_U_DIV ? 40u : 10u;
        }
        cost[s] = c;
    }
    std::vector<uint32_t> order(n_sets);
    for (size_t s = 0; s < n_sets; ++s) order[s] = (uint32_t)s;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        return wide[a] != wide[b] ? wide[a] < wide[b] : cost[a] > cost[b];
    });

    // One device block, one copy: [code | consts + one zero entry | schema | parents | descs |
    // order | scratch | found], each region 256-byte aligned (found[] right after the scratch's
    // counter lines, so a search reads both back in one copy, check_collect).  The zero entry past the
    // constant pool: the generator's constant gather is issued before it knows whether the
    // set has constants (pf_eval.hip gen_var), so a set with none reads the entry at its own
    // const_off, which may be the pool's end.
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    // the code region carries one zero instruction past the last END: the kernel fetches the
    // slot after an END before its dispatch leaves the program (pf_eval.hip run_program)
    const size_t o_code = 0, o_const = o_code + al(n_ins * 16 + 16), o_schema = o_const + al(n_const * 32 + 32),
                 o_par = o_schema + al(n_vars * 16), o_desc = o_par + al(n_parents * 32),
                 o_order = o_desc + al(n_sets * sizeof(pf_set_desc)), o_scr = o_order + al(n_sets * 4),
                 o_found = o_scr + PF_SCRATCH_BYTES,
                 total = o_found + al(std::max<size_t>(n_sets, 1) * 4);
    static_assert(PF_SCRATCH_BYTES % 256 == 0 && PF_COUNTER_OFF + PF_COUNTER_STRIPES * 128 == PF_SCRATCH_BYTES,
                  "found[] follows the counter lines");
    // scratch / found are cleared by every search: the copy ends at o_scr
    auto fill = [&](uint8_t* stage) {
        memset(stage, 0, o_scr);
        auto put = [&](size_t off, const void* src, size_t bytes) {
            if (bytes && src) memcpy(stage + off, src, bytes);
        };
        put(o_code, code, n_ins * 16);
        put(o_const, consts, n_const * 32);
        put(o_schema, schema, n_vars * 16);
        put(o_par, parents, n_parents * 32);
        put(o_desc, descs, n_sets * sizeof(pf_set_desc));
        put(o_order, order.data(), n_sets * 4);
    };

    // No g_mu from here on either: the device lookup holds g_devs_mu (pf_init and
    // pf_init_contexts insert under it; the Dev objects themselves never move), the block comes
    // from the pool under its own lock, errors go through t_err.
    Batch* B = nullptr;
    int dev_id = -1;
    hipStream_t ups = nullptr;
    auto report = [](int rc) {
        t_defer_err = false;
        std::lock_guard<std::mutex> lk(g_mu);
        g_err = t_err;
        return rc;
    };
    t_defer_err = true;
    {
        Dev* Dv = nullptr;
        {
            std::lock_guard<std::mutex> dk(g_devs_mu);
            Dv = use_dev(device);
        }
        if (!Dv) return report(-1);
        if (!handle_out) return report(fail("pf_batch_create: null handle_out"));
        B = new Batch();
        B->device = Dv->key;
        B->n_ins = n_ins;
        B->n_const = n_const;
        B->n_vars = n_vars;
        B->n_parents = n_parents;
        B->n_sets = n_sets;
        B->max_vars = max_vars;
        B->n_narrow = (size_t)std::count(wide.begin(), wide.end(), (uint8_t)0);
        // a set without variables counts as parented: its every candidate is candidate 0 (a
        // single query's ground keccak bucket left every such batch without the probe launch)
        B->all_parented = std::all_of(descs, descs + n_sets, [](const pf_set_desc& d) {
            return d.parent_off != PF_NO_PARENT || d.n_vars == 0;
        });
        B->h_descs.assign(descs, descs + n_sets);
        B->d_mem = pool_acquire(Dv, total, &B->mem_cap);
        if (!B->d_mem) {
            delete B;
            return report(fail("pf_batch_create: hipMalloc(%zu) failed", total));
        }
        uint8_t* base = static_cast<uint8_t*>(B->d_mem);
        B->d_code = reinterpret_cast<uint4*>(base + o_code);
        B->d_consts = reinterpret_cast<uint32_t*>(base + o_const);
        B->d_schema = reinterpret_cast<uint4*>(base + o_schema);
        B->d_parents = reinterpret_cast<uint32_t*>(base + o_par);
        B->d_descs = reinterpret_cast<pf_set_desc*>(base + o_desc);
        B->d_order = reinterpret_cast<uint32_t*>(base + o_order);
        B->d_found = reinterpret_cast<uint32_t*>(base + o_found);
        B->d_scratch = reinterpret_cast<uint32_t*>(base + o_scr);
        if (event_acquire(Dv, &B->ev0) != hipSuccess || event_acquire(Dv, &B->ev1) != hipSuccess) {
            const int rc = fail("pf_batch_create: hipEventCreate failed");
            release_batch(Dv, B);
            return report(rc);
        }
        dev_id = Dv->id;
        ups = Dv->up_stream;
    }
    t_defer_err = false;
    // the copy itself outside g_mu, on the device's upload stream through the upload staging
    // buffer (a search holding g_mu meanwhile runs on the library stream)
    bool ok = true;
    {
        std::lock_guard<std::mutex> lk(g_up_mu);
        ok = hipSetDevice(dev_id) == hipSuccess;
        uint8_t* pin = ok ? upload_staging(o_scr) : nullptr;
        if (pin) {
            fill(pin);
            ok = hipMemcpyAsync(B->d_mem, pin, o_scr, hipMemcpyHostToDevice, ups) == hipSuccess &&
                 hipStreamSynchronize(ups) == hipSuccess;
        } else if (ok) {
            std::vector<uint8_t> stage(o_scr);
            fill(stage.data());
            ok = hipMemcpy(B->d_mem, stage.data(), o_scr, hipMemcpyHostToDevice) == hipSuccess;
        }
    }
    if (!ok) {
        // the copy may still be in flight: drain the device and free the block rather than
        // pool it (the next pool_acquire would hand out memory still being written)
        t_defer_err = true;
        const int rc = fail("pf_batch_create: hipMemcpy of %zu bytes failed", o_scr);
        if (hipDeviceSynchronize() == hipSuccess) hipFree(B->d_mem);
        B->d_mem = nullptr;
        delete B;
        return report(rc);
    }
    *handle_out = (uint64_t)(uintptr_t)B;
    return 0;
}

int pf_batch_create(const uint32_t* code, size_t n_ins, const uint32_t* consts, size_t n_const,
                    const uint32_t* schema, size_t n_vars, const uint32_t* parents,
                    size_t n_parents, const pf_set_desc* descs, size_t n_sets,
                    uint64_t* handle_out) {
    return pf_batch_create_on(-1, code, n_ins, consts, n_const, schema, n_vars, parents, n_parents,
                              descs, n_sets, handle_out);
}

int pf_batch_free(uint64_t handle) {
    std::lock_guard<std::mutex> lk(g_mu);
    Batch* B = as_batch(handle);
    if (!B) return 0;
    Dev* D = use_dev(B->device);
#ifdef PF_FREE_DEVICE_SYNC
    hipDeviceSynchronize();
#else
    // a *_dev launch may still be reading the batch on a caller's stream: drain the stream of
    // the device's last launch (switch_stream has drained every earlier one; the library's
    // own launches are complete when their call returns, and the upload's copy when
    // pf_batch_create returned).  A whole-device synchronisation here cost every
    // single-query call a device-wide round trip.
    if (D && D->last_stream) hipStreamSynchronize(D->last_stream);
#endif
    if (D) D->last_stream = nullptr;
    release_batch(D, B);
    return 0;
}

static int found_to_host(Batch* B, const std::vector<uint32_t>& found, uint32_t* found_out,
                         uint8_t* sat_bitmap_out, pf_stats* stats) {
    uint64_t nsat = 0;
    if (sat_bitmap_out) memset(sat_bitmap_out, 0, (B->n_sets + 7) / 8);
    for (size_t s = 0; s < B->n_sets; s++) {
        if (found_out) found_out[s] = found[s];
        if (found[s] != 0xffffffffu) {
            nsat++;
            if (sat_bitmap_out) sat_bitmap_out[s / 8] |= (uint8_t)(1u << (s % 8));
        }
    }
    if (stats) stats->n_sat = nsat;
    return 0;
}

int pf_check_batch(uint64_t handle, uint64_t global_seed, uint32_t budget, uint32_t flags,
                   uint32_t timeout_ms, uint32_t* found_out, uint8_t* sat_bitmap_out,
                   pf_stats* stats) {
    std::lock_guard<std::mutex> lk(g_mu);
    Batch* B = as_batch(handle);
    if (!B) return fail("pf_check_batch: null batch");
    Dev* D = use_dev(B->device);
    if (!D || switch_stream(D, D->stream)) return -1;
    if (check_enqueue(B, global_seed, budget, flags, timeout_ms, B->d_found, D->stream)) return -1;
    std::vector<uint32_t> found;
    if (check_collect(B, D->stream, stats, &found)) return -1;
    return found_to_host(B, found, found_out, sat_bitmap_out, stats);
}

int pf_check_batches(const uint64_t* handles, size_t n, uint64_t global_seed, uint32_t budget,
                     uint32_t flags, uint32_t timeout_ms, uint32_t* found_out, pf_stats* stats) {
    std::lock_guard<std::mutex> lk(g_mu);
    // 1. enqueue every batch's search on its device's stream: devices run concurrently
    for (size_t i = 0; i < n; ++i) {
        Batch* B = as_batch(handles[i]);
        if (!B) return fail("pf_check_batches: null batch %zu", i);
        Dev* D = use_dev(B->device);
        if (!D || switch_stream(D, D->stream)) return -1;
        if (check_enqueue(B, global_seed, budget, flags, timeout_ms, B->d_found, D->stream)) return -1;
    }
    // 2. gather: verdicts concatenated in handle order
    size_t off = 0;
    for (size_t i = 0; i < n; ++i) {
        Batch* B = as_batch(handles[i]);
        Dev* D = use_dev(B->device);
        if (!D) return -1;
        pf_stats* st = stats ? stats + i : nullptr;
        std::vector<uint32_t> found;
        if (check_collect(B, D->stream, st, &found)) return -1;
        if (found_to_host(B, found, found_out ? found_out + off : nullptr, nullptr, st)) return -1;
        off += B->n_sets;
    }
    return 0;
}

int pf_check_batch_dev(uint64_t handle, uint64_t global_seed, uint32_t budget, uint32_t flags,
                       uint32_t timeout_ms, uint32_t* d_found, pf_stats* stats, void* stream) {
    std::lock_guard<std::mutex> lk(g_mu);
    Batch* B = as_batch(handle);
    if (!B) return fail("pf_check_batch_dev: null batch");
    if (!d_found) return fail("pf_check_batch_dev: null d_found");
    Dev* D = use_dev(B->device);
    if (!D) return -1;
    hipStream_t st = pick_stream(D, stream);
    if (switch_stream(D, st)) return -1;
    if (check_enqueue(B, global_seed, budget, flags, timeout_ms, d_found, st)) return -1;
    return stats ? check_collect(B, st, stats) : 0;
}

int pf_materialize(uint64_t handle, uint64_t global_seed, const uint32_t* set_ids,
                   const uint32_t* cand_ids, size_t n, uint32_t* values_out) {
    std::lock_guard<std::mutex> lk(g_mu);
    Batch* B = as_batch(handle);
    if (!B) return fail("pf_materialize: null batch");
    Dev* D = use_dev(B->device);
    if (!D) return -1;
    hipStream_t st = D->stream;
    if (n == 0) return 0;
    std::vector<uint32_t> off(n);
    uint64_t total = 0;
    for (size_t i = 0; i < n; i++) {
        if (set_ids[i] >= B->n_sets) return fail("pf_materialize: set %u out of range", set_ids[i]);
        off[i] = (uint32_t)total;
        total += B->h_descs[set_ids[i]].n_vars;
    }
    if (total == 0) return 0;
    if (switch_stream(D, st)) return -1;
    // one block from the device pool ([sets | cands | offsets | values], the index arrays
    // 256-byte aligned) and the pinned staging buffer for both copies: no hipMalloc / hipFree
    // (hipFree synchronises the device) and no pageable copies per call — this runs once per
    // funnel query whose witness is not a parented candidate 0
    const size_t o_in = ((3 * n * 4) + 255) & ~size_t(255), bytes = o_in + total * 32;
    size_t cap = 0;
    uint8_t* dm = static_cast<uint8_t*>(pool_acquire(D, bytes, &cap));
    if (!dm) return fail("pf_materialize: hipMalloc(%zu) failed", bytes);
    uint32_t *d_sets = reinterpret_cast<uint32_t*>(dm), *d_cands = d_sets + n, *d_off = d_cands + n,
             *d_out = reinterpret_cast<uint32_t*>(dm + o_in);
    uint8_t* pin = pinned_staging(std::max<size_t>(3 * n * 4, total * 32));
    int rc = 0;
    if (pin) {
        memcpy(pin, set_ids, n * 4);
        memcpy(pin + n * 4, cand_ids, n * 4);
        memcpy(pin + 2 * n * 4, off.data(), n * 4);
        if (hipMemcpyAsync(d_sets, pin, 3 * n * 4, hipMemcpyHostToDevice, st) != hipSuccess) rc = -1;
    } else if (hipMemcpyAsync(d_sets, set_ids, n * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
               hipMemcpyAsync(d_cands, cand_ids, n * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
               hipMemcpyAsync(d_off, off.data(), n * 4, hipMemcpyHostToDevice, st) != hipSuccess) {
        rc = -1;
    }
    if (!rc) {
        const uint32_t mv = std::max<uint32_t>(B->max_vars, 1u);
        const uint64_t threads = (uint64_t)n * mv;
        hipLaunchKernelGGL(pf_materialize_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0,
                           st, B->d_descs, B->d_code, B->d_consts, B->d_schema, B->d_parents,
                           global_seed, d_sets, d_cands, d_off, (uint32_t)n, mv, d_out);
        // the staging buffer is reused for the values: the stream orders the copies after the
        // kernel, which has consumed the index copy
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(pin ? static_cast<void*>(pin) : static_cast<void*>(values_out), d_out, total * 32,
                           hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            rc = -1;
    }
    if (!rc && pin) memcpy(values_out, pin, total * 32);
    if (rc) {
        // a failed copy or synchronisation after the copy-in may leave work on the stream
        // that still reads or writes the block: it is not pooled again — freed
        // after a full device synchronisation (whose own failure leaks it rather than hand
        // memory in use to the next pool_acquire)
        if (hipDeviceSynchronize() == hipSuccess) hipFree(dm);
        return fail("pf_materialize: HIP call failed");
    }
    // back to the pool (the stream is drained)
    pool_release(D, dm, cap);
    return 0;
}

static int eval_launch(Batch* B, uint32_t set, const uint32_t* d_soa, uint32_t n_cand,
                       uint8_t* d_out, hipStream_t st) {
    if (set >= B->n_sets) return fail("eval: set %u out of range", set);
    if (n_cand == 0) return 0;
    hipLaunchKernelGGL(pf_eval_soa_kernel, dim3((n_cand + 255) / 256), dim3(256), 0, st, B->d_descs,
                       set, B->d_code, B->d_consts, B->d_schema, B->d_parents, d_soa, n_cand, d_out);
    HIPCHK(hipGetLastError());
    return 0;
}

int pf_eval_assignments(uint64_t handle, uint32_t set, const uint32_t* soa, uint32_t n_cand,
                        uint8_t* sat_out) {
    std::lock_guard<std::mutex> lk(g_mu);
    Batch* B = as_batch(handle);
    if (!B) return fail("pf_eval_assignments: null batch");
    Dev* D = use_dev(B->device);
    if (!D) return -1;
    hipStream_t st = D->stream;
    if (set >= B->n_sets) return fail("eval: set %u out of range", set);
    if (n_cand == 0) return 0;
    const size_t nv = std::max<uint32_t>(B->h_descs[set].n_vars, 1u);
    const size_t bytes = nv * 8 * (size_t)n_cand * 4;
    if (switch_stream(D, st)) return -1;
    // one pooled block [assignments | verdicts] and the pinned staging buffer for both
    // copies (the GPU-resident ModelCache calls this once per quick-sat query: no hipMalloc /
    // hipFree, no pageable copies — pf_materialize's pattern)
    const size_t o_out = (bytes + 255) & ~size_t(255), total = o_out + n_cand;
    size_t cap = 0;
    uint8_t* dm = static_cast<uint8_t*>(pool_acquire(D, total, &cap));
    if (!dm) return fail("pf_eval_assignments: hipMalloc(%zu) failed", total);
    uint32_t* d_soa = reinterpret_cast<uint32_t*>(dm);
    uint8_t* d_out = dm + o_out;
    uint8_t* pin = pinned_staging(std::max<size_t>(bytes, n_cand));
    int rc = 0;
    if (pin) memcpy(pin, soa, bytes);
    if (hipMemcpyAsync(d_soa, pin ? static_cast<const void*>(pin) : static_cast<const void*>(soa), bytes,
                       hipMemcpyHostToDevice, st) != hipSuccess)
        rc = -1;
    if (!rc && eval_launch(B, set, d_soa, n_cand, d_out, st)) rc = -1;
    // the staging buffer is reused for the verdicts: the stream orders the copy after the
    // kernel, which ran after the copy-in
    if (!rc && (hipMemcpyAsync(pin ? static_cast<void*>(pin) : static_cast<void*>(sat_out), d_out, n_cand,
                               hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess))
        rc = -1;
    if (!rc && pin) memcpy(sat_out, pin, n_cand);
    if (rc) {
        // work may still be in flight on the block: freed after a full synchronisation, never
        // pooled (the pf_materialize rule)
        if (hipDeviceSynchronize() == hipSuccess) hipFree(dm);
        return fail("pf_eval_assignments: HIP call failed");
    }
    pool_release(D, dm, cap);
    return 0;
}

// pf_eval_program / pf_eval_programs: the program(s) validated and rewritten exactly as by
// pf_batch_create (prepare_program), one pooled block [code | consts + zero entry | schema |
// descs | assignments | verdicts] and one copy each way through the pinned staging buffer;
// the stream is synchronised, not the device (no batch object, no events): the quick-sat call
// of the GPU-resident ModelCache, once or twice per objective-free query
// (mythril_amd/model_cache.py)
static int eval_programs(const char* who, int device, const uint32_t* code, size_t n_ins, const uint32_t* consts,
                         size_t n_const, const uint32_t* schema, size_t n_vars, const pf_set_desc* descs,
                         size_t n_sets, const uint32_t* soa, uint32_t n_cand, uint8_t* sat_out) {
    Dev* D = use_dev(device);
    if (!D) return -1;
    if (n_cand == 0 || n_sets == 0) return 0;
    if (!code || !sat_out || !descs || (n_vars && !soa)) return fail("%s: null argument", who);
    if (n_sets > 65535) return fail("%s: %zu programs (at most 65535)", who, n_sets);
    std::vector<uint32_t> code_out;
    std::vector<pf_set_desc> descs_out;
    std::vector<uint8_t> wide;
    uint32_t max_vars = 0;
    if (prepare_program(code, n_ins, consts, n_const, schema, n_vars, 0, descs, n_sets, code_out, descs_out, wide,
                        max_vars))
        return -1;
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t nv = std::max<size_t>(n_vars, 1), n_dev = code_out.size() / 4, n_out = n_sets * (size_t)n_cand;
    const size_t soa_bytes = nv * 8 * (size_t)n_cand * 4;
    const size_t o_code = 0, o_const = al(n_dev * 16 + 16), o_schema = o_const + al(n_const * 32 + 32),  // + the pad slot
                 o_desc = o_schema + al(nv * 16), o_soa = o_desc + al(n_sets * sizeof(pf_set_desc)),
                 o_out = o_soa + al(soa_bytes), total = o_out + n_out;
    uint8_t* pin = pinned_staging(std::max<size_t>(o_out, n_out));
    if (!pin) return fail("%s: no pinned staging buffer", who);
    memset(pin, 0, o_out);
    memcpy(pin + o_code, code_out.data(), n_dev * 16);
    if (n_const) memcpy(pin + o_const, consts, n_const * 32);
    if (n_vars) memcpy(pin + o_schema, schema, n_vars * 16);
    memcpy(pin + o_desc, descs_out.data(), n_sets * sizeof(pf_set_desc));
    if (n_vars) memcpy(pin + o_soa, soa, soa_bytes);
    hipStream_t st = D->stream;
    if (switch_stream(D, st)) return -1;
    size_t cap = 0;
    uint8_t* dm = static_cast<uint8_t*>(pool_acquire(D, total, &cap));
    if (!dm) return fail("%s: hipMalloc(%zu) failed", who, total);
    int rc = 0;
    if (hipMemcpyAsync(dm, pin, o_out, hipMemcpyHostToDevice, st) != hipSuccess) rc = -1;
    if (!rc) {
        hipLaunchKernelGGL(pf_eval_soa_sets_kernel, dim3((n_cand + 63) / 64, (unsigned)n_sets), dim3(64), 0, st,
                           reinterpret_cast<const pf_set_desc*>(dm + o_desc),
                           reinterpret_cast<const uint4*>(dm + o_code), reinterpret_cast<const uint32_t*>(dm + o_const),
                           reinterpret_cast<const uint4*>(dm + o_schema),
                           reinterpret_cast<const uint32_t*>(dm + o_soa), n_cand, dm + o_out);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(pin, dm + o_out, n_out, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            rc = -1;
    }
    if (rc) {
        if (hipDeviceSynchronize() == hipSuccess) hipFree(dm);
        return fail("%s: HIP call failed", who);
    }
    memcpy(sat_out, pin, n_out);
    pool_release(D, dm, cap);
    return 0;
}

int pf_eval_program(int device, const uint32_t* code, size_t n_ins, const uint32_t* consts, size_t n_const,
                    const uint32_t* schema, size_t n_vars, const uint32_t* soa, uint32_t n_cand,
                    uint8_t* sat_out) {
    std::lock_guard<std::mutex> lk(g_mu);
    const pf_set_desc d0{0u, (uint32_t)n_ins, 0u, (uint32_t)n_const, 0u, (uint32_t)n_vars, 0u, PF_NO_PARENT};
    return eval_programs("pf_eval_program", device, code, n_ins, consts, n_const, schema, n_vars, &d0, 1, soa,
                         n_cand, sat_out);
}

int pf_eval_programs(int device, const uint32_t* code, size_t n_ins, const uint32_t* consts, size_t n_const,
                     const uint32_t* schema, size_t n_vars, const pf_set_desc* descs, size_t n_sets,
                     const uint32_t* soa, uint32_t n_cand, uint8_t* sat_out) {
    std::lock_guard<std::mutex> lk(g_mu);
    return eval_programs("pf_eval_programs", device, code, n_ins, consts, n_const, schema, n_vars, descs, n_sets,
                         soa, n_cand, sat_out);
}

int pf_eval_assignments_dev(uint64_t handle, uint32_t set, const uint32_t* d_soa,
                            uint32_t n_cand, uint8_t* d_sat_out, void* stream) {
    std::lock_guard<std::mutex> lk(g_mu);
    Batch* B = as_batch(handle);
    if (!B) return fail("pf_eval_assignments_dev: null batch");
    Dev* D = use_dev(B->device);
    if (!D) return -1;
    if (switch_stream(D, pick_stream(D, stream))) return -1;
    return eval_launch(B, set, d_soa, n_cand, d_sat_out, pick_stream(D, stream));
}

int pf_keccak256_batch(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out32) {
    std::lock_guard<std::mutex> lk(g_mu);
    Dev* D = use_dev(-1);
    if (!D) return -1;
    hipStream_t st = D->stream;
    if (n == 0) return 0;
    for (size_t i = 0; i < n; i++)
        if (offsets[i + 1] < offsets[i]) return fail("keccak: offsets not monotone at %zu", i);
    const uint64_t total = offsets[n];
    if (switch_stream(D, st)) return -1;
    // one pooled block [offsets | messages | digests] and one copy each way through the
    // pinned staging buffer (a concretisation call hashes a handful of preimages: three
    // hipMalloc / hipFree pairs and pageable copies were most of its latency)
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t o_off = 0, o_data = al((n + 1) * 8), o_out = o_data + al(total ? total : 8),
                 all = o_out + n * 32;
    size_t cap = 0;
    uint8_t* dm = static_cast<uint8_t*>(pool_acquire(D, all, &cap));
    if (!dm) return fail("pf_keccak256_batch: hipMalloc(%zu) failed", all);
    uint8_t* pin = pinned_staging(std::max<size_t>(o_out, n * 32));
    int rc = 0;
    if (pin) {
        memcpy(pin + o_off, offsets, (n + 1) * 8);
        if (total) memcpy(pin + o_data, data, total);
        if (hipMemcpyAsync(dm, pin, o_data + total, hipMemcpyHostToDevice, st) != hipSuccess) rc = -1;
    } else if (hipMemcpyAsync(dm + o_off, offsets, (n + 1) * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
               (total && hipMemcpyAsync(dm + o_data, data, total, hipMemcpyHostToDevice, st) != hipSuccess)) {
        rc = -1;
    }
    if (!rc) {
        hipLaunchKernelGGL(pf_keccak_var_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st,
                           dm + o_data, reinterpret_cast<const uint64_t*>(dm + o_off), (uint64_t)n, dm + o_out);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(pin ? static_cast<void*>(pin) : static_cast<void*>(out32), dm + o_out, n * 32,
                           hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            rc = -1;
    }
    if (rc) {
        if (hipDeviceSynchronize() == hipSuccess) hipFree(dm);
        return fail("pf_keccak256_batch: HIP call failed");
    }
    if (pin) memcpy(out32, pin, n * 32);
    pool_release(D, dm, cap);
    return 0;
}

int pf_keccak256_fixed_dev(const uint8_t* d_data, uint32_t len, size_t n, uint8_t* d_out32,
                           float* kernel_ms, void* stream) {
    std::lock_guard<std::mutex> lk(g_mu);
    Dev* D = use_dev(-1);
    if (!D) return -1;
    if (n == 0) return 0;
    hipStream_t st = pick_stream(D, stream);
    if (switch_stream(D, st)) return -1;
    HIPCHK(hipEventRecord(D->ev0, st));
    const bool fast = (len % 16u) == 0u && len < 136u && (((uintptr_t)d_data) & 15u) == 0u;
#ifdef PF_KECCAK_PERSIST
    if (fast && len == 64u) {
        // chip-filling persistent grid: PF_KECCAK_PERSIST 256-thread blocks per CU
        const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, (uint64_t)D->num_cus * PF_KECCAK_PERSIST);
        hipLaunchKernelGGL(pf_keccak_fixed64_persist_kernel, dim3((uint32_t)blocks), dim3(256), 0,
                           st, d_data, (uint64_t)n, d_out32);
    } else
#endif
#ifdef PF_KECCAK_ILP2
    if (fast)
        hipLaunchKernelGGL(pf_keccak_fixed2_kernel, dim3((uint32_t)(((n + 1) / 2 + 255) / 256)), dim3(256), 0,
                           st, d_data, len, (uint64_t)n, d_out32);
    else
#endif
    if (fast)
        hipLaunchKernelGGL(pf_keccak_fixed_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0,
                           st, d_data, len, (uint64_t)n, d_out32);
    else
        hipLaunchKernelGGL(pf_keccak_stride_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256),
                           0, st, d_data, len, (uint64_t)n, d_out32);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(D->ev1, st));
    if (kernel_ms) {
        HIPCHK(hipEventSynchronize(D->ev1));
        HIPCHK(hipEventElapsedTime(kernel_ms, D->ev0, D->ev1));
    }
    return 0;
}

}  // extern "C"
