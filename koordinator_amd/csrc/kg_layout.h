// kg_layout.h — device-resident layout of the node snapshot and pod batch (host + device view).
//
// Node snapshot: one 320-byte record per node (array of records, 256-byte aligned array base).
// The select kernel walks nodes in wave-uniform order, so a record is fetched with a handful of
// scalar (s_load_dwordx16) loads and every field lives in SGPRs while the 64 lanes evaluate 64
// different pods; NUMA zone tables are kept in a side array read only for NUMA-policy nodes.
// Pods: struct-of-arrays, one lane per pod (coalesced dwordx2 loads, loaded once per kernel).
#pragma once
#include <stdint.h>

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
    N_FLAGS, N_CPUSET, N_AMP_CPUSET, N_SPARE0,
    // reciprocals (IEEE double bit patterns) of the static divisors
    N_RCP_CPU, N_RCP_MEM, N_RCP_SC0, N_RCP_SC1, N_RCP_LA0, N_RCP_LA1,
    N_SPARE1, N_SPARE2,
    N_SLOTS
};
static_assert(N_SLOTS == 40, "node record is 40 x 8 bytes");

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
};
enum : uint32_t { FMODE_CHECK = 0, FMODE_PASS = 1, FMODE_FAIL_EXPIRED = 2 };

constexpr int MAX_ZONES = 4;
struct alignas(64) ZoneRec {
    int64_t cpu[MAX_ZONES], mem[MAX_ZONES], cpu_used[MAX_ZONES], mem_used[MAX_ZONES];
    double rcp_cpu[MAX_ZONES], rcp_mem[MAX_ZONES];
};

// Pod batch (device pointers, SoA). flags: low 16 bits KG_POD_*, bits 16..19 pod NUMA policy.
struct PodsDev {
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
};

// Scoring / filtering configuration passed by value to every kernel.
struct KCfg {
    uint32_t plugins;
    uint32_t la_score_enabled, la_score_prod, pad0;
    int64_t w_nrf, w_la, w_numa;
    int64_t nrf_w[4];  // cpu, memory, scalar0, scalar1
    int64_t la_w[2];
    int64_t la_dom_w;
    int64_t la_wsum;   // Σ la_w (+ dominant) — constant per profile
    int64_t numa_w_cpu, numa_w_mem, numa_hint_w_cpu, numa_hint_w_mem;
};

}  // namespace kg
