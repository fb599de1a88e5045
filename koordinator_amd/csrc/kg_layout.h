// kg_layout.h — device-resident layout of the node snapshot and pod batch (host + device view).
//
// Node snapshot: one 512-byte record per node. Slots [0, 40) are the authoritative int64 state
// (what Assume/Forget change); slots [40, 64) are exact float64 derivations of it ("headroom"
// values such as allocatable - requested) recomputed by derive_node() whenever the int state
// changes — on the host at upload and on the device after every Assume. The select kernel walks
// nodes in wave-uniform order, so a record arrives through the scalar cache (s_load_dwordx16) and
// lives in SGPRs while 64 lanes evaluate 64 different pods; NUMA zone tables are a side array read
// only for SingleNUMANode nodes.
// Pods: struct-of-arrays, one lane per pod (coalesced loads, once per kernel).
#pragma once
#include <stdint.h>
#include <string.h>

#include "../../include/koordgpu.h"

#if defined(__HIPCC__)
#define KG_HD __host__ __device__
#else
#define KG_HD
#endif

namespace kg {

enum NodeSlot : int {
    N_ALLOC_CPU = 0, N_ALLOC_MEM, N_ALLOC_EPH, N_ALLOC_PODS,
    N_REQ_CPU, N_REQ_MEM, N_REQ_EPH, N_NUM_PODS,
    N_NZ_CPU, N_NZ_MEM,
    N_SC_ALLOC0, N_SC_ALLOC1, N_SC_REQ0, N_SC_REQ1,
    N_LA_ALLOC0, N_LA_ALLOC1,
    N_LA_FCUT_NP0, N_LA_FCUT_NP1, N_LA_FCUT_PROD0, N_LA_FCUT_PROD1,
    N_LA_FBASE_NP0, N_LA_FBASE_NP1, N_LA_FBASE_PROD0, N_LA_FBASE_PROD1,
    N_LA_SBASE_NP0, N_LA_SBASE_NP1, N_LA_SBASE_PROD0, N_LA_SBASE_PROD1,
    N_CPUSET, N_AMP_CPUSET,
    N_RSV_CLASSES,        // Reservation: bit c set when the node has a restore view for owner class c
    N_DEV_MINORS,         // DeviceShare: GPU minors of the node's Device (-1: no Device object)
    N_INT_SLOTS,
    // ---- fast block [32, 64): read by the select kernel with wide scalar loads per node ----
    //  * N_FLAGS: low 32 bits device flags, high 32 bits the node's snapshot index (records are
    //    stored grouped by storage class, see node_class);
    //  * static slots (host, at upload; never touched by derive_node): upward-rounded reciprocals
    //    of the divisors and the plugin weights already masked by "capacity != 0";
    //  * derived slots (derive_node): headrooms x100 as exact float64 integers.
    FAST_BEGIN = 32,
    N_FLAGS = 32,
    // 1/capacity rounded toward +inf (0 for capacity 0): floor((F*100 - x*100) * rcp) is the exact
    // truncating quotient for 0 <= F <= capacity < 2^44 (see lr100 in kg_eval.h)
    N_RCP_CPU, N_RCP_MEM, N_RCP_SC0, N_RCP_SC1, N_RCP_LA0, N_RCP_LA1,
    N_W_NRF01,            // uint32 x 2: 2 x LeastAllocated weight of cpu, memory (0 if capacity 0)
    N_W_NRF23,            // uint16 x 2: same for scalar0, scalar1 | float 1 / max(Σ 2w of all four, 2)
    N_W_NUMA,             // uint32 2*w_cpu, uint32 2*w_mem of the NodeNUMAResource score (0 if capacity 0)
    N_W_AUX,              // float 0.5 / (w_cpu + w_mem) of the NUMA score | float 1 / max(N_W_NRF01 sum, 2)
    D_FIT_CPU,            // 100 * max(0, alloc - requested): Fits (pod request r fails iff 100 r > this)
    D_FIT_MEM, D_FIT_EPH, D_FIT_SC0, D_FIT_SC1,
    D_LR_NZ_CPU,          // 100 * (alloc - nonzero requested): LeastAllocated cpu
    D_LR_NZ_MEM,
    D_LR_SC0, D_LR_SC1,   // 100 * (alloc - requested) of the scalar resources
    D_LA_HEAD_NP0, D_LA_HEAD_NP1,      // 100 * (usage cut-off - filter base), non-prod / prod profile
    D_LA_HEAD_PROD0, D_LA_HEAD_PROD1,
    D_LA_SFREE_NP0, D_LA_SFREE_NP1,    // 100 * (LoadAware allocatable - non-prod score base)
    D_LA_SDELTA0, D_LA_SDELTA1,        // 100 * (non-prod score base - prod score base)
    D_NUMA_FREE_CPU,      // 100 * (alloc_cpu - requested_cpu): NodeNUMAResource score, no amplification
    D_NUMA_FREE_MEM,
    D_AMP_FIT,            // 100 * max(0, alloc_cpu - amplified requested): filterAmplifiedCPUs (2^62 if no amplification)
    D_AMP_DELTA,          // 100 * (requested - amplified requested): scoreWithAmplifiedCPUs (0 if no amplification)
    N_SLOTS
};
static_assert(N_INT_SLOTS == 32, "int section is 32 x 8 bytes");
static_assert(N_SLOTS == 64, "node record is 64 x 8 bytes");

// The fast block as the select kernel sees it (a by-value copy -> wide scalar loads).
struct alignas(64) FastRec {
    int64_t flags;  // low: flags, high: snapshot index
    double rcp_cpu, rcp_mem, rcp_sc0, rcp_sc1, rcp_la0, rcp_la1;
    uint64_t w_nrf01, w_nrf23, w_numa, w_aux;
    double fit_cpu, fit_mem, fit_eph, fit_sc0, fit_sc1;
    double lr_nz_cpu, lr_nz_mem, lr_sc0, lr_sc1;
    double la_head_np0, la_head_np1, la_head_prod0, la_head_prod1;
    double la_sfree_np0, la_sfree_np1, la_sdelta0, la_sdelta1;
    double numa_free_cpu, numa_free_mem, amp_fit, amp_delta;
};
static_assert(sizeof(FastRec) == 8 * (N_SLOTS - FAST_BEGIN), "fast block layout");

struct alignas(64) NodeRec {
    int64_t v[N_SLOTS];
};

// Device flag word (NodeRec.v[N_FLAGS])
enum : uint32_t {
    F_LA_FMODE_NP_SHIFT = 0,   // 2 bits: LoadAware filter mode for non-prod pods
    F_LA_FMODE_PROD_SHIFT = 2, // 2 bits: for prod pods
    F_LA_NP_AGG = 1u << 4,     // non-prod profile is the aggregated-usage profile (reason text)
    F_LA_PROD_THR = 1u << 5,   // prod pods use the prod profile
    F_LA_SCORE_ZERO = 1u << 6, // LoadAware Score returns 0 (no metric / expired / NodeMetric nil)
    F_LA_HAS_METRIC = 1u << 7, // podAssignCache holds the node's NodeMetric (Reserve updates bases)
    F_NUMA_POLICY_SHIFT = 8,   // 4 bits KG_NUMA_*
    F_NUMA_ZONES_SHIFT = 12,   // 4 bits zone count
    F_AMP = 1u << 16,          // cpu amplification ratio > 1
    F_PODS_FULL = 1u << 17,    // len(Pods) + 1 > AllowedPodNumber (derived)
    F_BIG = 1u << 18,          // some value is outside the exact float64 fast path (derived)
    F_TOPO = 1u << 19,         // BestEffort node: Filter / Score like policy None, the Reserve runs the topology
                               // manager (window replay takes the integer path for the Reserve's zone)
    F_VBIG = 1u << 20,         // F_BIG for a value outside the fast path (not only for the node's policies): the fast
                               // block's NodeResourcesFit / LoadAware part is exact unless this is set (derived)
    F_RSV_NUMA = 1u << 21,     // a reservation on the node holds a NUMA / cpuset allocation (kg_node_columns.rsv_numa):
                               // pairs whose NodeNUMAResource reads its restore are KG_ST_UNSUPPORTED
    F_DERIVED_MASK = F_PODS_FULL | F_BIG | F_VBIG,
};
enum : uint32_t { FMODE_CHECK = 0, FMODE_PASS = 1, FMODE_FAIL_EXPIRED = 2 };

constexpr int MAX_ZONES = 4;
// Fast view of one NUMA zone (select kernel, SingleNUMANode class): derived headrooms x100 plus
// static reciprocals / masked weights set by the host at upload.
struct alignas(16) ZoneFast {
    double avail_cpu, avail_mem;  // 100 * max(0, total - used); -1 when that is 0 (never eligible)
    double hint_cpu, hint_mem;    // 100 * (total - max(0, total - available)): hint-score headroom
    double free_cpu, free_mem;    // 100 * (total - used): allocation-score headroom
    double rcp_cpu, rcp_mem;      // static: 1/total rounded toward +inf (0 if total 0)
    uint64_t w_hint;              // static: uint32 2*hint_w_cpu, 2*hint_w_mem (0 if total 0)
    uint64_t w_score;             // static: uint32 2*w_cpu, 2*w_mem (0 if total 0)
    uint64_t hpack;               // static: float 0.5/(hint weights), float 0.5/(score weights)
};
struct alignas(64) ZoneRec {
    int64_t cpu[MAX_ZONES], mem[MAX_ZONES], cpu_used[MAX_ZONES], mem_used[MAX_ZONES];
    double rcp_cpu[MAX_ZONES], rcp_mem[MAX_ZONES];
    ZoneFast zf[MAX_ZONES];
    uint32_t status;  // NUMANodeSharedStatus, 2 bits per zone (0 idle, 1 single, 2 shared)
    uint32_t pad_;
    double amp_ratio;  // cpu amplification ratio (filterAmplifiedCPUs amplifies a cpuset-binding pod's request)
    // cpuset binding (kg_cpuset.h): topology index (-1: none), packed meta (CPU_META_*), and the counts the
    // Filter compares numCPUsNeeded with, derived from the node's kg_cpu_alloc (cpu_counts)
    int32_t cpu_topo;
    uint32_t cpu_meta;
    int32_t cpu_free;        // CPUs with RefCount < maxRefCount (getAvailableCPUs)
    int32_t cpu_free_full;   // of those, the CPUs of cores whose every CPU is free (required FullPCPUs)
    int32_t cpu_free_cores;  // cores with a free CPU (required SpreadByPCPUs: one CPU per core)
    int32_t cpu_allocated;   // CPUs with RefCount > 0 (cpuset_alloc_milli / 1000)
    // DeviceShare GPU topology of the node (static; kg_node_columns.dev_topo / dev_part): per minor
    // (NUMA rank << 4 | PCIe rank) or KG_GPU_NO_SCOPE, and the partition table / KG_GPU_HONOR / KG_GPU_TREE
    uint64_t dev_topo;
    uint32_t dev_part;
    // per minor (nibble) the GPU's NUMA node id, KG_GPU_NUMA_ANY (NodeID -1) or KG_GPU_NUMA_NONE (no Topology):
    // DeviceShare as a NUMA hint provider (kg_node_columns.dev_numa)
    uint32_t dev_numa;
    // per NUMA node (cpu_counts): available CPUs (RefCount < maxRefCount), of those the CPUs of whole free cores
    // (required FullPCPUs), the cores with a free CPU (required SpreadByPCPUs), and the allocated CPUs (RefCount > 0,
    // the amplified zone accounting of zone_cpu_alloc)
    uint16_t cz_free[MAX_ZONES], cz_full[MAX_ZONES], cz_cores[MAX_ZONES], cz_alloc[MAX_ZONES];
    // per NUMA node the cpuset pods in NodeAllocation.singleNUMANode / sharedNode (node_allocation.go:111-143): the
    // statuses (bits 0-7 of status) follow from them, and a cpuset Release takes its pod out again
    // (kg_node_columns.numa_zone_pods; saturating at 255)
    uint8_t cz_single[MAX_ZONES], cz_shared[MAX_ZONES];
};
static_assert(sizeof(ZoneRec) == 704, "ZoneRec: zones, fast zone view, cpuset counts, GPU topology");
// ZoneRec.status bit ZONE_RECORD_SHIFT + z: zone z holds an allocatedResources record (kg_node_columns.numa_zone_status)
constexpr uint32_t ZONE_RECORD_SHIFT = KG_ZONE_RECORD_SHIFT;

// extension.Amplify: ceil(v * ratio) for ratio > 1
KG_HD inline int64_t amp_i64(int64_t v, double ratio) {
#ifdef __HIP_DEVICE_COMPILE__
    return ratio > 1.0 ? (int64_t)ceil(__dmul_rn((double)v, ratio)) : v;
#else
    return ratio > 1.0 ? (int64_t)ceil((double)v * ratio) : v;
#endif
}

// NodeAllocation.getAvailableNUMANodeResources (node_allocation.go:221-243): the cpu allocated in zone q as the topology
// manager counts it; on an amplified node a zone with an allocation record counts its cpuset CPUs amplified
KG_HD inline int64_t zone_cpu_alloc(const ZoneRec& z, uint32_t q) {
    const int64_t u = z.cpu_used[q];
    if (!((z.status >> (ZONE_RECORD_SHIFT + q)) & 1u) || !(z.amp_ratio > 1.0)) return u;
    const int64_t cs = 1000 * (int64_t)z.cz_alloc[q];
    return u - cs + amp_i64(cs, z.amp_ratio);
}
// ZoneRec.cpu_meta: bits 0-7 maxRefCount, 8-9 node CPU bind policy (KG_NODE_CPU_BIND_*), 10 NUMA allocate
// strategy, 11-14 CPUs per core
constexpr uint32_t CPU_META_BIND_SHIFT = 8, CPU_META_STRATEGY_SHIFT = 10, CPU_META_CPC_SHIFT = 11;

// The Filter's view of a node's allocated CPUs (ZoneRec.cpu_free / cpu_free_full / cpu_free_cores /
// cpu_allocated), recomputed on the host at upload and on the device after a cpuset Reserve.
KG_HD inline __attribute__((always_inline)) void cpu_counts(const kg_cpu_topo& t, const kg_cpu_alloc* a, int max_ref, ZoneRec& z) {
    int free_core[KG_MAX_CPUS], core_numa[KG_MAX_CPUS];
    for (int k = 0; k < t.n_cores; k++) free_core[k] = 0, core_numa[k] = 0;
    int fr = 0, al = 0;
    int zfree[MAX_ZONES] = {0, 0, 0, 0}, zalloc[MAX_ZONES] = {0, 0, 0, 0};
    for (int c = 0; c < t.n_cpus; c++) {
        const int ref = a ? a->ref[c] : 0;
        const int q = t.numa[c];
        core_numa[t.core[c]] = q;
        if (ref < max_ref) {
            fr++;
            free_core[t.core[c]]++;
            if (q < MAX_ZONES) zfree[q]++;
        }
        al += ref > 0;
        if (ref > 0 && q < MAX_ZONES) zalloc[q]++;
    }
    // filterCPUsByRequiredCPUBindPolicy counts a core for FullPCPUs when its free CPUs number CPUsPerCore()
    const int cpc = t.n_cores ? t.n_cpus / t.n_cores : 0;
    int full = 0, cores = 0;
    int zfull[MAX_ZONES] = {0, 0, 0, 0}, zcores[MAX_ZONES] = {0, 0, 0, 0};
    for (int k = 0; k < t.n_cores; k++) {
        full += free_core[k] == cpc ? cpc : 0;
        cores += free_core[k] > 0;
        const int q = core_numa[k];  // a core lies in one NUMA node
        if (q < MAX_ZONES) {
            zfull[q] += free_core[k] == cpc ? cpc : 0;
            zcores[q] += free_core[k] > 0;
        }
    }
    z.cpu_free = fr;
    z.cpu_free_full = full;
    z.cpu_free_cores = cores;
    z.cpu_allocated = al;
    for (int q = 0; q < MAX_ZONES; q++) {
        z.cz_free[q] = (uint16_t)zfree[q];
        z.cz_full[q] = (uint16_t)zfull[q];
        z.cz_cores[q] = (uint16_t)zcores[q];
        z.cz_alloc[q] = (uint16_t)zalloc[q];
    }
}

// NUMANodeSharedStatus (node_allocation.go:60-68) from the zone's single / shared pod counts: shared if any shared pod
// is there, single if only single pods, idle if none; the other status bits (allocation records) are kept. Status bits
// cover zones < MAX_ZONES.
KG_HD inline uint32_t zone_status_of_counts(const ZoneRec& z) {
    uint32_t st = z.status & ~0xFFu;
    for (uint32_t q = 0; q < (uint32_t)MAX_ZONES; q++)
        st |= (z.cz_shared[q] ? 2u : z.cz_single[q] ? 1u : 0u) << (2 * q);
    return st;
}

// Zone code of a pair whose Reserve fails (BestEffort allocation): 0x20 | KG_ST_NUMA_INSUF_* >> 12.
constexpr int32_t ZONE_RESERVE_FAIL = 0x20;
KG_HD inline bool zone_reserve_fails(int32_t z) { return z >= 0x20 && z < 0x40; }
// a cpuset-binding pod whose accumulator finds no CPUs at Reserve (resource_manager.go:385,427 ErrNotEnoughCPUs)
constexpr int32_t ZONE_CPUSET_FAIL = ZONE_RESERVE_FAIL | 8;
// a GPU pod whose DeviceShare hints or Allocate fail in the topology manager at Reserve (BestEffort node):
// ZONE_GPU_FAIL | KG_DEV_CODE_*, or ZONE_GPU_FAIL | 0xF for "Reservation(s) Insufficient gpu devices"
constexpr int32_t ZONE_GPU_FAIL = 0x30;
KG_HD inline int32_t zone_gpu_fail(uint32_t st) {
    return ZONE_GPU_FAIL | (int32_t)((st & KG_ST_DEV_RSV) ? 0xFu : KG_ST_DEV_CODE(st));
}
KG_HD inline uint32_t zone_fail_status(int32_t z) {
    if ((uint32_t)z & 0x10u) return ((z & 0xF) == 0xF) ? (uint32_t)KG_ST_DEV_RSV : KG_ST_DEV_MAKE((uint32_t)z & 0xFu);
    return (((uint32_t)z & 7u) << 12) | (((uint32_t)z & 8u) ? KG_ST_NUMA_CPUS : 0u);
}
// Reserve of one (pod, node): the zone code the pre-Reserve state gives, handed from the kernel that evaluates it
// (k_ext_assume's evaluation pass, k_cpuset_reserve) to the one that applies (k_assume / k_ext_assume) in the
// pair's out word, so that the cpuset take in between does not change the pair's Reserve (zone codes fit a byte)
constexpr int32_t ZONE_PRESET = 0x40000000;
KG_HD inline int32_t zone_preset(int32_t z) { return ZONE_PRESET | (z & 0xFF); }
KG_HD inline bool zone_is_preset(int32_t w) { return (w & ZONE_PRESET) != 0; }
KG_HD inline int32_t zone_of_preset(int32_t w) { return (int32_t)(int8_t)(uint8_t)(w & 0xFF); }
// the NUMA affinity (bit per zone) of a pair's zone code; 0 = none (nil affinity, or the Reserve fails)
KG_HD inline uint32_t zone_affinity(int32_t z) {
    if (z < 0 || zone_reserve_fails(z)) return 0u;
    return z >= 0x40 ? ((uint32_t)z & 0xFu) : (1u << (uint32_t)z);
}

// Magnitude bound of the float64 fast path: operands below 2^44 keep 100 * headroom below 2^51
// (exact) and make the upward-rounded reciprocal's quotient exact after truncation.
constexpr int64_t FAST_LIMIT = (int64_t)1 << 44;

KG_HD inline bool kg_big(int64_t x) { return x >= FAST_LIMIT || x <= -FAST_LIMIT; }

KG_HD inline int64_t kg_bits(double d) {
    int64_t b;
    memcpy(&b, &d, 8);
    return b;
}

KG_HD inline double x100(int64_t x) { return (double)x * 100.0; }  // exact for |x| < 2^46

KG_HD inline uint32_t node_index(const NodeRec& r) { return (uint32_t)((uint64_t)r.v[N_FLAGS] >> 32); }

// Recompute the derived section of a node record (flags F_PODS_FULL / F_BIG, headrooms, zone
// headrooms) from its int section. Used by the host runtime at upload and by the device after
// Assume/Forget, so both sides produce identical bits. Static slots are left alone.
KG_HD inline void derive_node(NodeRec& r, ZoneRec& z) {
    int64_t* v = r.v;
    uint32_t f = (uint32_t)v[N_FLAGS] & ~(uint32_t)F_DERIVED_MASK;
    if (v[N_NUM_PODS] + 1 > v[N_ALLOC_PODS]) f |= F_PODS_FULL;
    // F_BIG: some operand is outside the fast path (magnitude >= 2^44, or a negative quantity,
    // which could push a headroom above its capacity); such nodes take the integer path
    bool big = false;
    for (int s = N_ALLOC_CPU; s <= N_LA_SBASE_PROD1; s++) {
        if (s == N_ALLOC_PODS || s == N_NUM_PODS) continue;
        if (s >= N_LA_FCUT_NP0 && s <= N_LA_FCUT_PROD1) continue;  // cut-offs may be INT64_MAX or -1
        big = big || kg_big(v[s]) || v[s] < 0;
    }
    big = big || kg_big(v[N_CPUSET]) || kg_big(v[N_AMP_CPUSET]) || v[N_CPUSET] < 0 || v[N_AMP_CPUSET] < v[N_CPUSET];
    for (uint32_t q = 0; q < (uint32_t)MAX_ZONES; q++) {
        const int64_t tc = z.cpu[q], tm = z.mem[q], uc = zone_cpu_alloc(z, q), um = z.mem_used[q];
        big = big || kg_big(tc) || kg_big(tm) || kg_big(uc) || kg_big(um) || z.cpu_used[q] < 0 || um < 0;
        const int64_t ac = tc - uc < 0 ? 0 : tc - uc, am = tm - um < 0 ? 0 : tm - um;
        const int64_t rc = tc - ac < 0 ? 0 : tc - ac, rm = tm - am < 0 ? 0 : tm - am;
        ZoneFast& zf = z.zf[q];
        zf.avail_cpu = ac != 0 ? x100(ac) : -1.0;
        zf.avail_mem = am != 0 ? x100(am) : -1.0;
        zf.hint_cpu = x100(tc - rc);
        zf.hint_mem = x100(tm - rm);
        zf.free_cpu = x100(tc - uc);
        zf.free_mem = x100(tm - um);
    }
    if (big) f |= F_VBIG;
    // Restricted nodes run the general NUMA topology manager in Filter, on the integer path (BestEffort
    // nodes do not admit in Filter, plugin.go:446-455: their Filter / Score fit the fast path)
    const uint32_t pol0 = (f >> F_NUMA_POLICY_SHIFT) & 15u;
    big = big || pol0 == 2u /* KG_NUMA_RESTRICTED */;
    // a node CPU bind policy makes every pod with a cpu request bind cpusets there (util.go:121-138)
    big = big || ((z.cpu_meta >> CPU_META_BIND_SHIFT) & 3u) != 0u;
    // a NUMA policy on a node whose reservations hold NUMA / cpuset allocations: the integer path reports the pairs
    big = big || ((f & F_RSV_NUMA) && pol0 != 0u /* KG_NUMA_NONE */);
    if (big) f |= F_BIG;
    v[N_FLAGS] = (int64_t)(((uint64_t)v[N_FLAGS] & 0xFFFFFFFF00000000ull) | f);
    auto fit = [](int64_t x) { return kg_bits(x100(x < 0 ? 0 : x)); };
    const int64_t always_fail = kg_bits(-1.0);  // below every fast-path request (requests are >= 0)
    const int64_t never_fail = kg_bits(4611686018427387904.0);  // 2^62: above every fast-path request
    // "Too many pods" folded into the cpu check: every pod then fails it
    v[D_FIT_CPU] = (f & F_PODS_FULL) ? always_fail : fit(v[N_ALLOC_CPU] - v[N_REQ_CPU]);
    v[D_FIT_MEM] = fit(v[N_ALLOC_MEM] - v[N_REQ_MEM]);
    v[D_FIT_EPH] = fit(v[N_ALLOC_EPH] - v[N_REQ_EPH]);
    v[D_FIT_SC0] = fit(v[N_SC_ALLOC0] - v[N_SC_REQ0]);
    v[D_FIT_SC1] = fit(v[N_SC_ALLOC1] - v[N_SC_REQ1]);
    v[D_LR_NZ_CPU] = kg_bits(x100(v[N_ALLOC_CPU] - v[N_NZ_CPU]));
    v[D_LR_NZ_MEM] = kg_bits(x100(v[N_ALLOC_MEM] - v[N_NZ_MEM]));
    v[D_LR_SC0] = kg_bits(x100(v[N_SC_ALLOC0] - v[N_SC_REQ0]));
    v[D_LR_SC1] = kg_bits(x100(v[N_SC_ALLOC1] - v[N_SC_REQ1]));
    // cut-offs may be INT64_MAX ("no check"): the float64 difference stays >= 2^53 there, above any
    // fast-path estimate, and is exact everywhere else
    // The profile's filter mode is folded into the heads: PASS -> 2^62 (never over), FAIL_EXPIRED -> -1
    // (always over); nodes without prod thresholds give prod pods the non-prod heads.
    auto head = [&](uint32_t mode, int64_t cut, int64_t base) {
        return mode == FMODE_PASS ? never_fail
             : mode == FMODE_FAIL_EXPIRED ? always_fail : kg_bits(((double)cut - (double)base) * 100.0);
    };
    const uint32_t m_np = (f >> F_LA_FMODE_NP_SHIFT) & 3u, m_pr = (f >> F_LA_FMODE_PROD_SHIFT) & 3u;
    v[D_LA_HEAD_NP0] = head(m_np, v[N_LA_FCUT_NP0], v[N_LA_FBASE_NP0]);
    v[D_LA_HEAD_NP1] = head(m_np, v[N_LA_FCUT_NP1], v[N_LA_FBASE_NP1]);
    const bool prod_thr = (f & F_LA_PROD_THR) != 0;
    v[D_LA_HEAD_PROD0] = prod_thr ? head(m_pr, v[N_LA_FCUT_PROD0], v[N_LA_FBASE_PROD0]) : v[D_LA_HEAD_NP0];
    v[D_LA_HEAD_PROD1] = prod_thr ? head(m_pr, v[N_LA_FCUT_PROD1], v[N_LA_FBASE_PROD1]) : v[D_LA_HEAD_NP1];
    v[D_LA_SFREE_NP0] = kg_bits(x100(v[N_LA_ALLOC0] - v[N_LA_SBASE_NP0]));
    v[D_LA_SFREE_NP1] = kg_bits(x100(v[N_LA_ALLOC1] - v[N_LA_SBASE_NP1]));
    v[D_LA_SDELTA0] = kg_bits(x100(v[N_LA_SBASE_NP0] - v[N_LA_SBASE_PROD0]));
    v[D_LA_SDELTA1] = kg_bits(x100(v[N_LA_SBASE_NP1] - v[N_LA_SBASE_PROD1]));
    v[D_NUMA_FREE_CPU] = kg_bits(x100(v[N_ALLOC_CPU] - v[N_REQ_CPU]));
    v[D_NUMA_FREE_MEM] = kg_bits(x100(v[N_ALLOC_MEM] - v[N_REQ_MEM]));
    // filterAmplifiedCPUs: requested' = requested - cs + Amplify(cs) when requested >= cs > 0
    const int64_t req = v[N_REQ_CPU], cs = v[N_CPUSET], acs = v[N_AMP_CPUSET];
    const int64_t req_f = (req >= cs && cs > 0) ? req - cs + acs : req;
    const bool amp = (f & F_AMP) != 0;
    // Restricted nodes are outside the fast path (F_BIG): every non-skipped pod fails here
    const uint32_t pol = (f >> F_NUMA_POLICY_SHIFT) & 15u;
    const bool pol_host = pol == 2u /* KG_NUMA_RESTRICTED */;
    v[D_AMP_FIT] = pol_host ? always_fail : amp ? fit(v[N_ALLOC_CPU] - req_f) : never_fail;
    // scoreWithAmplifiedCPUs: requested - cs + Amplify(cs) unconditionally under policy None; a BestEffort
    // node scores node allocatable / requested as they are (calculateAllocatableAndRequested, scoring.go:184-189)
    v[D_AMP_DELTA] = kg_bits((amp && pol != 1u /* KG_NUMA_BEST_EFFORT */) ? x100(cs - acs) : 0.0);
}

// Storage class of a node record: the select kernel is specialised per class and the snapshot is
// stored grouped by class (class 0 first), each group in ascending snapshot order.
KG_HD inline int node_class(const NodeRec& r) {
    return (((uint32_t)r.v[N_FLAGS] >> F_NUMA_POLICY_SHIFT) & 15u) == 3u /* KG_NUMA_SINGLE_NODE */ ? 1 : 0;
}

// Pod flag bit 20 (set by the host): every request value is inside the float64 fast domain (the pod may still take
// the integer lanes for its NUMA policy or cpuset binding): its NodeResourcesFit / LoadAware fast part is exact.
constexpr uint32_t POD_FASTV = 1u << 20;

// Pod batch (device pointers, SoA). flags: low 16 bits KG_POD_*, bits 16..19 pod NUMA policy, bit 20 POD_FASTV.
struct PodsDev {
    // config-5 columns (nullptr unless the snapshot enables DeviceShare / Reservation / ElasticQuota)
    const int64_t* dev_req;     // [pod][KG_DEV_R]
    const uint32_t* dev_count;
    const uint32_t* dev_keys;
    const int32_t* quota;
    const uint32_t* quota_keys;
    const int32_t* rsv_class;
    const int64_t* req_cpu;
    const int64_t* req_mem;
    const int64_t* req_eph;
    const int64_t* sc_req0;
    const int64_t* sc_req1;
    const int64_t* nz_cpu;
    const int64_t* nz_mem;
    const int64_t* la_est0;
    const int64_t* la_est1;
    const uint32_t* flags;
    const uint8_t* dev_cls;     // GPU request class of the pod (DevSum.code / score index), DEV_CLASSES = none
    const uint32_t* dev_flags;  // KG_GPU_POD_*
    const int64_t* dev_bw;      // ring bus bandwidth request (KG_GPU_POD_RING_BW)
    const uint32_t* dev_tmpl;   // candidate template counts per key (KG_GPU_POD_TEMPLATE)
};

// Scoring / filtering configuration passed by value to every kernel.
// Weights are host-validated to [0, 2^20] so int32 holds them (fewer SGPRs in the select loop).
struct KCfg {
    uint32_t plugins;
    uint32_t la_score_enabled, la_score_prod;
    int32_t w_nrf, w_la, w_numa;
    int32_t nrf_w[4];  // cpu, memory, scalar0, scalar1
    int32_t la_w[2];
    int32_t la_dom_w;
    int32_t la_wsum;   // Σ la_w + dominant weight — constant per profile
    int32_t numa_w_cpu, numa_w_mem, numa_hint_w_cpu, numa_hint_w_mem;
    float la_hw;       // 0.5 / la_wsum (0 when la_wsum is 0): fast-path weighted quotient
    int32_t w_dev, w_rsv;
    int32_t dev_w[3];  // DeviceShare LeastAllocated weights {gpu-core, gpu-memory-ratio, gpu-memory}
    uint32_t most;     // MostAllocated strategies: bit 0 NUMA score, bit 1 NUMA hint score, bit 2 DeviceShare
    uint32_t nrf_most; // NodeResourcesFit MostAllocated resources: bit r of {cpu, memory, scalar0, scalar1}
    uint32_t nrf_ign, rsv_ign;  // scalars left out of NodeResourcesFit Fits / Reservation fitsNode (bit k)
};
enum : uint32_t { MOST_NUMA = 1u, MOST_NUMA_HINT = 2u, MOST_DEV = 4u };

// ---- config-5 side tables (integer path) -----------------------------------------------------------
constexpr int DEV_MINORS = 8, DEV_R = 3;
// DeviceShare minors of one node record (side array in record order).
struct alignas(64) DevRec {
    int64_t total[DEV_R][DEV_MINORS];
    int64_t free_[DEV_R][DEV_MINORS];
};

// Per-(pod batch, node record) DeviceShare summary (k_dev_sum): the pod batch's distinct GPU requests
// (at most DEV_CLASSES, host-assigned per pod) each get the GPU allocator's outcome on the record
// (gpu_allocate's reason code) and the node Score, so that the config-5 fast path does not run the
// allocator or walk the minors per pair.
constexpr int DEV_CLASSES = 56;
// A GPU request class: everything the allocator reads of a pod (GPURequirements).
struct DevClass {
    int64_t dreq[DEV_R];
    uint32_t dkeys, dcount, dflags, dtmpl;
    int64_t dbw;
};
struct alignas(16) DevSum {
    int64_t T[DEV_R], F[DEV_R];
    double rcp[DEV_R];             // 1 / T (least_req's exact-quotient path)
    uint8_t code[DEV_CLASSES];     // per class: the GPU allocator's DeviceShare reason code (0 = the pod fits)
    uint8_t score[DEV_CLASSES];    // per class: the node Score (scoreNode over the minor sums, 0..100) of one instance
};
constexpr int QUOTA_R = 4;
// ElasticQuota mutable state (double-buffered during replay) and static limits.
struct alignas(16) QuotaState {
    int64_t used[QUOTA_R], np_used[QUOTA_R];
    uint32_t used_keys, np_keys;
    uint64_t pad_;
};
struct alignas(16) QuotaLim {
    int64_t limit[QUOTA_R], min[QUOTA_R];
    uint32_t limit_keys, min_keys;
    uint64_t pad_;
};

constexpr int RSV_R = 5, RSV_MAX_CLASSES = 64, RSV_MAX_PER_VIEW = 8;
// Reservation restore view (kg_rsv_view with the node's record position).
struct alignas(16) RsvView {
    uint32_t rec, first, count, cls;
    int64_t req[RSV_R];
    int64_t nz_cpu, nz_mem, num_pods;
    int64_t pod_requested[RSV_R];
    int64_t r_allocated[RSV_R];
    int32_t dev_base;  // DevRec of the restore's allocation outside the reservations (-1: the node's)
    uint32_t pad_;
};
struct alignas(16) RsvInfo {
    uint32_t policy, names, allocate_once;
    int32_t dev;  // DevRec a pod allocates from this reservation (-1: it reserves no GPU)
    int64_t order;
    int64_t allocatable[RSV_R], allocated[RSV_R], reserved[RSV_R];
    int64_t max_pods, allocated_pods;
    uint32_t rid, allocated_keys;  // kg_rsv_info.rid / .allocated_keys
    uint32_t dev_pref;             // kg_rsv_info.dev_minors: the reserved GPU minors, taken first
    uint32_t pad_;
    uint64_t pad2_;
};

// Replay with reservation views: per step (ring of 3) the pairs whose Reservation score term can be nonzero (a
// nominated reservation's score or a reservation order), its maximum and the preferred-node key, and the step's
// winner (picked by the step launch's last workgroup).
struct alignas(16) RsvStep {
    uint64_t win;   // winning key of the step (0 = none)
    uint64_t pref;  // min pref_key over the feasible pairs with an order (~0 = none)
    uint32_t cnt;   // entries in the step's list
    uint32_t rmax;  // max nominated-reservation score over the feasible pairs
};

// DeviceShare restore inputs of the nodes whose reservations hold GPUs (kg_rsv_gpu): the node's raw used
// (nodeDevice.deviceUsed) and its GPU-holding reservations [first, first + count) of GpuRawRsv; per reservation the
// reserve pod's allocation, its assigned pods' allocations on those minors, policy and assigned pod count. A GPU pod's
// Reserve on such a node updates them and rebuilds the node's restore tables (gpu_restore_rebuild, kg_ext.h).
struct alignas(16) GpuRawNode {
    int64_t used[DEV_R][DEV_MINORS];
    uint32_t first, count;
    uint64_t pad_;
};
struct alignas(16) GpuRawRsv {
    int64_t alloc[DEV_R][DEV_MINORS];
    int64_t allocated[DEV_R][DEV_MINORS];
    uint32_t rid, policy;
    int64_t pods;
};

// Device pointers of the config-5 tables of a snapshot (nullptr when the plugin is off).
struct ExtDev {
    const DevRec* dev;             // [record]
    const QuotaLim* qlim;          // [quota]
    QuotaState* qstate;            // [2][quota] (replay double buffer; outside replay both agree)
    uint32_t n_quotas;
    const RsvView* views;          // sorted by class, then record position
    const RsvInfo* infos;
    const uint32_t* cls_begin;     // [RSV_MAX_CLASSES + 1] view range per class
    // direct view lookup: the record's views in class order are vmap[vfirst[rec] + k] (k = the rank of the class among
    // the record's N_RSV_CLASSES bits), each an index into views
    const uint32_t* vfirst;        // [record]
    const uint32_t* vmap;          // [view]
    const DevRec* rdev;            // GPU restore tables of views / reservations (kg_rsv_dev)
    const DevSum* dsum;            // [record] of the current pod batch (fast-base select / stats only)
    // Fast-base select of the GPU pods in one pass (k_ext_select<FB>): the DeviceShare maximum over the fast-base
    // records is taken as cls_max[class] (the class's best score over every fast-base record whose allocator
    // succeeds: an upper bound, k_dev_sum), the real one goes to fb_max[pod]; k_ext_fix_rows lists the rows
    // whose guess was wrong and the same kernel re-runs them (rows[0, *n_rows)) with the final maximum.
    const uint32_t* cls_max;  // [DEV_CLASSES]; nullptr = dev_max is final
    uint32_t* fb_max;         // [pod]
    const uint32_t* rows;     // nullptr = every row
    const uint32_t* n_rows;
    uint32_t rows_from;       // the launch's first pod block takes rows[rows_from ...]
    // GPU partition tables (kg_gpu_partition, grouped by table / GPU count / AllocationScore) and per (table,
    // GPU count) the entry range: part_rng[table * 9 + n] = begin | end << 16
    const kg_gpu_partition* parts;
    uint32_t n_parts;
    const uint32_t* part_rng;
    const int64_t* binpack;  // [table][8, 4, 2 GPUs][allocated minors]: free partitions' AllocationScore sum
    // per batch (with dsum): the GPU allocator's code of every restore table (rdev) for every GPU request class,
    // [table][DEV_CLASSES]; nullptr = run the allocator
    const uint8_t* rcode;
    // per batch (with dsum): DeviceShare's contribution to the topology manager of the class-1 (SingleNUMANode)
    // records, [record - n0][DEV_CLASSES] (gpu_zone_sum); nullptr = evaluate those records on the general path
    const uint64_t* gz;
    // GPU-holding reservations (kg_snapshot_upload_rsv_gpu): per record its GpuRawNode (-1 = none; nullptr = no node
    // has one), the nodes' and reservations' raw restore inputs
    const int32_t* graw;
    GpuRawNode* gnodes;
    GpuRawRsv* grsv;
    // fast-base config-5 batch: the general pairs' selection inputs, stored by the statistics pass
    // (k_ext_stats_sp: a GPU pod's every general pair; k_ext_stats_views: a class pod's views) for the select pass
    // (k_ext_select_sp), [position][xpos[pod]] (position: the pair's rank in for_general_records, < xT; xpos: the pod's
    // lane in the select pass's list, xn lanes; nullptr = the pod's batch index): neighbouring lanes of both passes
    // store and load neighbouring words
    // (XPAIR_*); nullptr = none
    uint64_t* xpairs;
    uint32_t xT, xn;
    const uint32_t* xpos;
    const uint32_t* xsp;  // the special list the positions count from (k_special_scan)
};

}  // namespace kg
