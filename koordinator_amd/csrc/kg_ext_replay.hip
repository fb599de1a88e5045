// kg_ext_replay.hip — CDNA4 (gfx950) config-5 replay step (k_ext_replay: one pod per launch, lane = node record,
// the previous pod's Reserve applied in place, the launch's last workgroup picks the winner) and the single-pod
// Reserve / Unreserve (k_ext_assume). Split from kg_ext.hip so the translation units compile in parallel.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kg_cpuset_reserve.h"
#include "kg_ext.h"
#include "kg_ext_wave.h"
#include "kg_kernels.h"

namespace kg {

// Winner of pod `step` (one wave: the last workgroup of the step's launch, after every other workgroup evaluated the
// pod): NormalizeScore of DeviceShare from the score buckets (M = the highest raw score among the feasible nodes; a
// bucket's key is base total << 32 | index, so key(b) = base + w_dev * 100 s / M) and, with reservation views, of
// Reservation (the listed pairs' maximum, or 1000 and the preferred node at 1000 when a reservation order exists,
// total_ext). A pair off the list has a zero Reservation term, so its bucket key is its total; a listed pair's bucket
// key is a lower bound of its total: the maximum over the buckets and the list is the winner.
__device__ __forceinline__ uint64_t ext_replay_pick(uint32_t step, uint32_t n_nodes, const KCfg& cfg,
                                                    const uint64_t* __restrict__ buckets, const RsvStep* __restrict__ rs,
                                                    const uint64_t* __restrict__ rlist) {
    const uint32_t lane = threadIdx.x;
    const uint64_t* B = buckets + (size_t)(step % 3) * 128 * REPLAY_BUCKET_STRIDE;
    const uint64_t b0 = ld_agent(B + lane * REPLAY_BUCKET_STRIDE), b1 = ld_agent(B + (lane + 64) * REPLAY_BUCKET_STRIDE);
    const int32_t M = wmax_i32(max(b0 ? (int32_t)lane : -1, b1 ? (int32_t)lane + 64 : -1));
    if (M < 0) return 0ull;  // no feasible node (a listed pair is also in its bucket)
    auto cand = [&](uint64_t b, int64_t sd) -> uint64_t {
        if (!b) return 0ull;
        const int64_t tot = (int64_t)(b >> 32) + (int64_t)cfg.w_dev * norm100(sd, M);
        return ((uint64_t)tot << 32) | (b & 0xFFFFFFFFull);
    };
    const uint64_t c0 = cand(b0, lane), c1 = cand(b1, lane + 64);
    uint64_t best = c0 > c1 ? c0 : c1;
    if (rs) {
        const RsvStep& z = rs[step % 3];
        const uint64_t pf = ld_agent(&z.pref);
        const uint32_t rmax = ld_agent(&z.rmax), cnt = ld_agent(&z.cnt);
        const int64_t rm = pf != PREF_NONE ? 1000 : (int64_t)rmax;
        const uint64_t* L = rlist + (size_t)(step % 3) * n_nodes * 2;
        // the listed pairs, U entries per lane in flight per round trip (a class pod lists up to its class's views)
        constexpr uint32_t U = 8;
        for (uint32_t k0 = 0; k0 < cnt; k0 += 64u * U) {
            uint64_t kb[U], sc[U];
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                const uint32_t k = k0 + u * 64u + lane;
                kb[u] = k < cnt ? ld_agent(L + 2 * (size_t)k) : 0ull;
                sc[u] = k < cnt ? ld_agent(L + 2 * (size_t)k + 1) : 0ull;
            }
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                const uint32_t g = 0xFFFFFFFFu - (uint32_t)(kb[u] & 0xFFFFFFFFull);
                const int64_t sd = (int64_t)(uint32_t)(sc[u] >> 32);
                const int64_t rsv = (pf != PREF_NONE && (uint32_t)pf == g) ? 1000 : (int64_t)(uint32_t)sc[u];
                const int64_t tot =
                    (int64_t)(kb[u] >> 32) + (int64_t)cfg.w_dev * norm100(sd, M) + (int64_t)cfg.w_rsv * norm100(rsv, rm);
                const uint64_t key = kb[u] ? (((uint64_t)tot << 32) | (kb[u] & 0xFFFFFFFFull)) : 0ull;
                best = key > best ? key : best;
            }
        }
    }
    return wmax_u64(best);
}

// Arrival of a workgroup (one lane, after the workgroup's barrier) on the launch's counters (REPLAY_DONE_*): true in
// the last workgroup to arrive. One counter for every workgroup serialises their atomics (~19 us a launch for 1.6k
// workgroups); workgroup b arrives on shard b % REPLAY_DONE_SHARDS, the last of each shard on the top counter. Every
// counter is back at 0 when the launch ends.
__device__ __forceinline__ bool last_arrival(uint32_t* done) {
    const uint32_t G = gridDim.x, sh = blockIdx.x % REPLAY_DONE_SHARDS;
    const uint32_t n_sh = G < REPLAY_DONE_SHARDS ? G : REPLAY_DONE_SHARDS;
    const uint32_t in_sh = (G - sh + REPLAY_DONE_SHARDS - 1u) / REPLAY_DONE_SHARDS;  // workgroups of shard sh
    uint32_t* c = done + (size_t)(1u + sh) * REPLAY_DONE_STRIDE;
    if (atomicAdd(c, 1u) != in_sh - 1u) return false;
    st_agent(c, 0u);  // every workgroup of the shard has arrived
    if (atomicAdd(done, 1u) != n_sh - 1u) return false;
    st_agent(done, 0u);
    return true;
}

// A pair of a fast-base replay (FB: every pod in the fast domain, the three base plugins, DeviceShare read from the
// batch's DevSum table, the SingleNUMANode records' GPU hints from e.gz) on the fast block, as the fast-base select
// evaluates it (k_ext_select<FB>, eval_c1): the key (base total << 32 | ~g, 0 = infeasible), DeviceShare's raw score and
// the Reserve's zone. false: the pair takes eval_pair_ext (F_BIG, a view of the pod's reservation class, a BestEffort
// record whose Reserve zone comes from the topology manager, an unclassed GPU pod).
__device__ __forceinline__ bool replay_fast_pair(const KCfg& cfg, const KCfg& cv, const ExtDev& e, const int64_t* __restrict__ n,
                                                 const ZoneRec* __restrict__ zr, uint32_t rec, uint32_t n0, const PodF& pff,
                                                 const PodX& px, uint32_t dcls, bool off, uint32_t g, uint64_t& kb,
                                                 int32_t& s_dev, int32_t& zone) {
    const uint32_t fl = (uint32_t)n[N_FLAGS];
    if (fl & F_BIG) return false;
    if ((cfg.plugins & KG_PLUGIN_RSV) && px.cls >= 0 && px.cls < RSV_MAX_CLASSES &&
        (((uint64_t)n[N_RSV_CLASSES] >> px.cls) & 1ull))
        return false;
    const bool dev = (cfg.plugins & KG_PLUGIN_DEV) && px.dcount != 0;
    if (dev && dcls >= (uint32_t)DEV_CLASSES) return false;
    const FastRec fr = *reinterpret_cast<const FastRec*>(&n[FAST_BEGIN]);
    uint64_t bk;
    int64_t sd = 0;
    uint32_t st;
    zone = -1;
    if (rec < n0) {
        if (((fl >> F_NUMA_POLICY_SHIFT) & 15u) != (uint32_t)KG_NUMA_NONE) return false;
        bk = eval_fast_key<7u, 0>(cv, fr, zr, pff, g);
        st = (bk == 0ull || off) ? 1u : 0u;
        if (!st && dev) st = dev_eval_cls(n, e.dsum + rec, px, dcls, sd);
    } else if (dev) {
        if (!e.gz) return false;
        const uint64_t gz = e.gz[(size_t)(rec - n0) * DEV_CLASSES + dcls];
        bk = eval_fast_key<7u, 1, true>(cv, fr, zr, pff, g, &zone, gz);
        st = (bk == 0ull || off) ? 1u : 0u;
        if (!st) {
            if (zone >= 0 && !(gz & GZ_NODEV)) {  // DeviceShare's Allocate under the admitted zone, its Score there
                st = ((gz >> (12 + zone)) & 1ull) ? 0u : 1u;
                sd = (int64_t)((gz >> (16 + 8 * zone)) & 0xFFull);
            } else {
                st = dev_eval_cls(n, e.dsum + rec, px, dcls, sd);
            }
        }
    } else {
        bk = eval_fast_key<7u, 1>(cv, fr, zr, pff, g, &zone);
        st = (bk == 0ull || off) ? 1u : 0u;
    }
    if (st) zone = -1;
    kb = st ? 0ull : bk;
    s_dev = (int32_t)sd;
    return true;
}

// The winner's DevSum entry (and its e.gz words on a SingleNUMANode record) after a Reserve that changed its minors, by
// the winner's whole wave (lane = GPU request class).
__device__ __forceinline__ void replay_refresh(const KCfg& cfg, const ExtDev& e, NodeRec* __restrict__ nodes,
                                               ZoneRec* __restrict__ zones, DevRec* __restrict__ devs, uint32_t r, uint32_t n0,
                                               const DevClass* __restrict__ dclass, uint32_t n_dclass) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the winner lane's minors stores, before the wave reads them
    dev_sum_refresh(cfg, e, nodes[r].v, zones + r, devs + r, dclass, n_dclass, const_cast<DevSum*>(e.dsum) + r);
    if (e.gz && r >= n0) {
        const uint32_t nc = min(n_dclass, (uint32_t)DEV_CLASSES);
        for (uint32_t k = threadIdx.x & 63u; k < nc; k += 64u) {
            PodX x{};
            x.dkeys = dclass[k].dkeys;
            x.dcount = dclass[k].dcount;
            x.dflags = dclass[k].dflags;
            x.dtmpl = dclass[k].dtmpl;
            x.dbw = dclass[k].dbw;
            for (int q = 0; q < DEV_R; q++) x.dreq[q] = dclass[k].dreq[q];
            const_cast<uint64_t*>(e.gz)[(size_t)(r - n0) * DEV_CLASSES + k] =
                gpu_zone_sum(cfg, e, nodes[r].v, zones + r, devs + r, x);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the entries, before the winner lane's evaluation reads them
}

// Reserve of pod q (step - 1) on its winner record i by the record's lane (the zone code of its pair: prev_zone, its
// nominated reservation in nsel): NodeInfo, LoadAware, NUMA zone, GPU minors, Reservation and DeviceShare bookkeeping.
// Returns whether the record's minors changed (its DevSum / e.gz entries are refreshed next).
__device__ __forceinline__ bool replay_reserve(const KCfg& cfg, const ExtDev& e, NodeRec* __restrict__ nodes,
                                            ZoneRec* __restrict__ zones, DevRec* __restrict__ devs, const PodsDev& pods,
                                            uint32_t q_idx, uint32_t i, int32_t prev_zone, int32_t nom_in,
                                            uint32_t* __restrict__ minors_out) {
    const PodV q = load_pod(pods, q_idx);
    const PodX qx = load_podx(pods, q_idx);
    const bool refresh = e.dsum && (cfg.plugins & KG_PLUGIN_DEV) && (qx.dcount > 0 || (e.graw && e.graw[i] >= 0));
    apply_assume(cfg, nodes[i].v, zones + i, q, prev_zone, 1);
    const int32_t nom = (nom_in >= 0 && nodes[i].v[N_RSV_CLASSES] != 0) ? nom_in : -1;
    uint32_t mask = 0;
    if ((cfg.plugins & KG_PLUGIN_DEV) && qx.dcount > 0) {
        mask = dev_choose_site(cfg, e, nodes[i].v, zones + i, devs + i, pod_view(cfg, e, nodes[i].v, i, qx), nom, qx,
                               prev_zone);
        *minors_out = mask;
    }
    // Reservation.Reserve into the nominated reservation, then DeviceShare's (the node's minors, or the restore inputs
    // and tables of GPU-holding reservations)
    if ((cfg.plugins & KG_PLUGIN_RSV) && nom_in != -2 && nodes[i].v[N_RSV_CLASSES] != 0)
        rsv_reserve_dev(e, nodes[i].v, zones + i, i, q, nom);
    dev_reserve_apply(cfg, e, nodes[i].v, i, devs + i, mask, qx, nom >= 0 ? (int32_t)e.infos[nom].rid : -1, 1);
    return refresh;
}

template <bool EXACT>
__device__ __forceinline__ PairX replay_general_pair(const KCfg& cfg, const ExtDev& e, const int64_t* __restrict__ n,
                                                  const ZoneRec* __restrict__ zr, const DevRec* d, uint32_t rec,
                                                  const PodV& p, const PodX& px, uint32_t dcls) {
    return eval_pair_ext<EXACT>(cfg, e, n, zr, d, rec, p, px, 0u, dcls);
}

// One replay step (see file header). buckets: [3][128] ring of per-DeviceShare-score best keys (REPLAY_BUCKET_STRIDE). winners[step - 1] holds
// the key the previous launch picked for pod step - 1; the winner record's lane applies its Reserve unless it fails
// (zone code of its pair, or a cpuset Reserve that failed in between, k_cpuset_reserve), every lane evaluates pod `step`
// on its record, then gates it on its quota. The last workgroup to finish (done counter) then picks pod step's winner into winners[step] and settles
// winners[step - 1] (0 when its Reserve failed): no other launch per step.
template <bool EXACT, bool FB>
__global__ __launch_bounds__(REPLAY_WG, 2) void k_ext_replay(NodeRec* __restrict__ nodes, ZoneRec* __restrict__ zones,
                                                   DevRec* __restrict__ devs, ExtDev e, PodsDev pods, uint32_t n_pods,
                                                   uint32_t n_nodes, uint32_t index_base, KCfg cfg,
                                                   const uint32_t* __restrict__ step_base, uint32_t step_off,
                                                   uint64_t* __restrict__ winners, uint32_t* __restrict__ minors,
                                                   uint64_t* __restrict__ buckets, int8_t* __restrict__ zsel,
                                                   uint32_t* __restrict__ reason, const uint32_t* __restrict__ pos,
                                                   int32_t* __restrict__ nsel, RsvStep* __restrict__ rs,
                                                   uint64_t* __restrict__ rlist, uint32_t* __restrict__ done,
                                                   const DevClass* __restrict__ dclass, uint32_t n_dclass, uint32_t n0) {
    const uint32_t step = (step_base ? *step_base : 0u) + step_off;
    if (step > n_pods) return;  // uniform
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t i = blockIdx.x * REPLAY_WG + threadIdx.x;
    // the workgroup's per-score-bucket maxima (one global atomic per bucket and workgroup)
    __shared__ uint64_t lb[128];
    for (uint32_t t = threadIdx.x; t < 128u; t += REPLAY_WG) lb[t] = 0ull;
    const bool live = i < n_nodes;
    const bool has_next = step < n_pods;
    const uint64_t prev = step > 0 ? __hip_atomic_load(&winners[step - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    const uint32_t gprev = 0xFFFFFFFFu - (uint32_t)(prev & 0xFFFFFFFFull);
    if (blockIdx.x == 0 && threadIdx.x < 64u) {
        uint64_t* Z = buckets + (size_t)((step + 1) % 3) * 128 * REPLAY_BUCKET_STRIDE;  // last read by the pick of step - 2
        Z[lane * REPLAY_BUCKET_STRIDE] = 0;
        Z[(lane + 64) * REPLAY_BUCKET_STRIDE] = 0;
        if (rs && lane == 0) {  // slot of step + 1 (last read by the pick of step - 2)
            RsvStep& z = rs[(step + 1) % 3];
            z.win = 0;
            z.pref = PREF_NONE;
            z.cnt = 0;
            z.rmax = 0;
        }
    }
    // Reserve of pod step-1 on its winner, by the winner record's lane. It fails (BestEffort NUMA allocation, or a
    // cpuset Reserve that failed between the launches) on the zone code of its pair: the pod stays unscheduled. zsel is
    // double-buffered by step parity: the previous step's codes are read while this step's are written.
    bool refresh = false;  // the winner's minors changed: its DevSum entry is refreshed below
    if (live && prev != 0ull && gprev == index_base + node_index(nodes[i])) {
        const int32_t prev_zone = zsel[(size_t)((step - 1) & 1u) * n_nodes + i];
        if (!zone_reserve_fails(prev_zone)) {
            // the nominated reservation of the winning pair (nsel, double-buffered like zsel); -2: no Reservation.Reserve
            const int32_t nom = ((cfg.plugins & KG_PLUGIN_RSV) && nsel) ? nsel[(size_t)((step - 1) & 1u) * n_nodes + i] : -2;
            refresh = replay_reserve(cfg, e, nodes, zones, devs, pods, step - 1, i, prev_zone, nom, minors + step - 1);
        }
    }
    if (const uint64_t own = __ballot(refresh))  // uniform per wave: the winner's workgroup
        replay_refresh(cfg, e, nodes, zones, devs, (i - lane) + (uint32_t)(__ffsll((unsigned long long)own) - 1), n0,
                       dclass, n_dclass);
    // pod `step` on every record, before its ElasticQuota gate (a uniform verdict applied below: the pair loads do not
    // wait for the previous Reserve's outcome)
    const PodV p = load_pod(pods, has_next ? step : 0);
    const PodX px = load_podx(pods, has_next ? step : 0);
    uint64_t kb = 0;
    int32_t s = 0;
    uint32_t stat = 0;
    if (has_next) {  // the final step only applies the last Reserve
        bool fast = false;
        if constexpr (FB) {  // the fast-base pairs (uniform per step: the pod's fast-path operands)
            const PodF pff = to_podf(p, cfg);
            const KCfg cv = cfg_in_vgprs(cfg);
            const bool off = (cfg.plugins & KG_PLUGIN_RSV) && (p.flags & KG_POD_RSV_REQUIRED);
            const uint32_t dcls = pods.dev_cls ? (uint32_t)pods.dev_cls[step] : (uint32_t)DEV_CLASSES;
            int32_t zone = -1;
            if (live) fast = replay_fast_pair(cfg, cv, e, nodes[i].v, zones + i, i, n0, pff, px, dcls, off,
                                              index_base + node_index(nodes[i]), kb, s, zone);
            if (fast) {
                zsel[(size_t)(step & 1u) * n_nodes + i] = (int8_t)zone;
                if (nsel) nsel[(size_t)(step & 1u) * n_nodes + i] = -1;
            }
        }
        if (live && !fast) {
            const uint32_t dcls = (e.dsum && pods.dev_cls) ? (uint32_t)pods.dev_cls[step] : (uint32_t)DEV_CLASSES;
            const PairX r = replay_general_pair<EXACT>(cfg, e, nodes[i].v, zones + i, devs ? devs + i : nullptr, i, p, px, dcls);
            zsel[(size_t)(step & 1u) * n_nodes + i] = (int8_t)r.zone;
            if (nsel) nsel[(size_t)(step & 1u) * n_nodes + i] = r.nom;
            stat = r.status;
            if (!r.status) {
                const int64_t base = (int64_t)cfg.w_nrf * r.s_nrf + (int64_t)cfg.w_la * r.s_la + (int64_t)cfg.w_numa * r.s_numa;
                const uint32_t g = index_base + node_index(nodes[i]);
                kb = ((uint64_t)base << 32) | (uint64_t)(0xFFFFFFFFu - g);
                s = (int32_t)r.s_dev;
                if (rs && (r.s_rsv != 0 || r.order != 0)) {
                    // a pair whose Reservation score term can be nonzero: listed for the pick (its bucket entry stays, a
                    // lower bound of its total)
                    RsvStep& z = rs[step % 3];
                    const uint32_t at = atomicAdd(&z.cnt, 1u);
                    st_agent(rlist + ((size_t)(step % 3) * n_nodes + at) * 2, kb);
                    st_agent(rlist + ((size_t)(step % 3) * n_nodes + at) * 2 + 1,
                             ((uint64_t)(uint32_t)r.s_dev << 32) | (uint32_t)r.s_rsv);
                    if (r.s_rsv) atomicMax(&z.rmax, (uint32_t)r.s_rsv);
                    if (r.order != 0) atomicMin((unsigned long long*)&z.pref, (unsigned long long)pref_key(r.order, g));
                }
            }
        }
    }
    // the previous Reserve's outcome, from the zone code of the winner's pair (the same word in every lane)
    bool placed1 = false;
    if (prev != 0ull) {
        const int32_t pz = zsel[(size_t)((step - 1) & 1u) * n_nodes + pos[gprev - index_base]];
        placed1 = !zone_reserve_fails(pz);
        if (!placed1 && blockIdx.x == 0 && threadIdx.x == 0 && reason) atomicOr(reason + step - 1, zone_fail_status(pz));
    }
    // ElasticQuota: buffer (step-1)&1 holds the state after pods < step-1; buffer step&1 becomes the
    // state after pods < step (block 0, nobody reads it during this launch). winners[step - 2] was settled by the last
    // workgroup of the previous launch.
    uint32_t qst = 0;
    if (cfg.plugins & KG_PLUGIN_QUOTA) {
        const uint32_t nq = e.n_quotas;
        const QuotaState* rd = e.qstate + (size_t)((step - 1) & 1u) * nq;
        PodX x1;
        PodV p1;
        if (step > 0) {
            p1 = load_pod(pods, step - 1);
            x1 = load_podx(pods, step - 1);
        }
        if (has_next && px.quota >= 0 && (uint32_t)px.quota < nq) {
            QuotaState S = rd[px.quota];
            if (placed1 && x1.quota == px.quota) quota_add(S, p1, x1, 1);
            qst = quota_gate(e.qlim[px.quota], S, p, px);
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            QuotaState* wr = e.qstate + (size_t)(step & 1u) * nq;
            if (step > 1 && winners[step - 2] != 0ull) {
                const PodV p2 = load_pod(pods, step - 2);
                const PodX x2 = load_podx(pods, step - 2);
                if (x2.quota >= 0 && (uint32_t)x2.quota < nq) quota_add(wr[x2.quota], p2, x2, 1);
            }
            if (placed1 && x1.quota >= 0 && (uint32_t)x1.quota < nq) quota_add(wr[x1.quota], p1, x1, 1);
        }
    }
    if (has_next) {
        if (qst) {  // PreFilter rejected the pod: no node is evaluated (eval_pair_ext's status)
            kb = 0ull;
            stat = live ? qst : 0u;
        }
        if (reason) {  // FitError diagnosis: OR of the filter status bits over the nodes
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) stat |= (uint32_t)__shfl_xor((int)stat, off, 64);
            if (lane == 0 && stat) atomicOr(reason + step, stat);
        }
        // per-score-bucket maxima: the workgroup's in LDS, then one global atomic per non-empty bucket (the score
        // buckets of a shared-GPU pod hold many distinct scores: per-wave global atomics serialise on their lines)
        __syncthreads();  // lb zeroed
        if (kb != 0ull) atomicMax((unsigned long long*)(lb + s), (unsigned long long)kb);
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < 128u; t += REPLAY_WG)
            if (lb[t] != 0ull)
                atomicMax((unsigned long long*)(buckets + ((size_t)(step % 3) * 128 + t) * REPLAY_BUCKET_STRIDE),
                          (unsigned long long)lb[t]);
    }
    // the last workgroup of the launch: pick pod step's winner, settle pod step-1's. The hand-off follows
    // MI355X_MICROARCH.md's "Consumer, always" form, the producers need no agent release: every byte the pick reads
    // was written by an agent-scope atomic or an sc1 (write-through) store (condition 2), every wave drains them
    // (vmcnt(0)) before the workgroup barrier behind which its first lane arrives (condition 3); the arrival that
    // completes the launch is the consumer's poll, followed by ONE agent-scope acquire in the picking wave only, then
    // sc1 loads (ext_replay_pick: ld_agent). The acquire is kept because the two-level arrival (a shard counter, then
    // the top counter for the whole shard) matches no single row of the guide's sc1 hand-off table (condition 4): row 1
    // grants "the last adder decides" to ONE unsharded counter only, and one counter for every workgroup serialises
    // ~1.6k atomics (~19 us a launch). Producers pay nothing; the picking wave pays one L1 invalidate (~1.7 us).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int last;
    if (threadIdx.x == 0) last = last_arrival(done) ? 1 : 0;
    __syncthreads();
    if (!last || threadIdx.x >= 64u) return;  // uniform per workgroup / per wave: the first wave picks
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the invalidate has completed before the pick's loads
    if (has_next) {
        const uint64_t w = qst ? 0ull : ext_replay_pick(step, n_nodes, cfg, buckets, rs, rlist);
        if (lane == 0) winners[step] = w;
    }
    if (lane == 0 && step > 0 && prev != 0ull && !placed1) winners[step - 1] = 0ull;  // the Reserve failed: unscheduled
}

// Reserve (sign +1: zone and minors chosen here, or preset in out by an evaluation pass) / Unreserve (sign -1: the
// given zone and minors). sign 0: the evaluation pass alone, which presets out for a cpuset Reserve and the Reserve.
// out: [0] zone, [1] minors, [2] nominated reservation (index into e.infos), [3] its rid (-1 = none).
// split (nullable): the NUMA allocation's per-zone amounts (cpu, then memory), written by a Reserve (zeroed by the
// caller; a cpuset Reserve under a NUMA affinity wrote them already) and given back by an Unreserve with the zone code
// 0x40 | mask. rsv: Reservation.Reserve / Unreserve on the node's views (an Unreserve into the reservation rid_in).
// cpus (Unreserve, nullable): the cpuset CPUs to release (NodeAllocation.release).
template <bool EXACT>
__global__ void k_ext_assume(NodeRec* __restrict__ nodes, ZoneRec* __restrict__ zones, DevRec* __restrict__ devs, ExtDev e,
                             PodsDev pods, uint32_t pod, uint32_t rec, int32_t zone_in, uint32_t minors_in, int64_t sign,
                             KCfg cfg, int32_t* __restrict__ out, int64_t* __restrict__ split, bool rsv, int32_t rid_in,
                             kg_cpu_alloc* __restrict__ allocs, const kg_cpu_topo* __restrict__ topos,
                             const uint64_t* __restrict__ cpus) {
    if (blockIdx.x != 0) return;
    // the whole wave evaluates (uniform work on a full exec mask), lane 0 applies
    const PodV q = load_pod(pods, pod);
    const PodX qx = load_podx(pods, pod);
    int64_t* n = nodes[rec].v;
    int32_t zone = zone_in;
    uint32_t mask = minors_in;
    int32_t nom = -1;
    if (sign >= 0 && out && zone_is_preset(out[0])) {
        // the evaluation pass ran before the cpuset Reserve (which may have failed it): zone, minors and nominated
        // reservation of the pre-take state
        zone = zone_of_preset(out[0]);
        mask = (uint32_t)out[1];
        nom = out[2];
        if (zone_reserve_fails(zone)) {
            if (threadIdx.x == 0) out[0] = zone, out[1] = 0;
            return;
        }
    } else if (sign >= 0) {
        const PairX r = eval_pair_ext<EXACT>(cfg, e, n, zones + rec, devs ? devs + rec : nullptr, rec, q, qx, 0u);
        zone = r.status ? -1 : r.zone;
        nom = r.status ? -1 : r.nom;
        if (zone_reserve_fails(zone)) {  // the NodeNUMAResource Reserve fails: nothing is applied
            if (out && threadIdx.x == 0) {
                out[0] = sign == 0 ? zone_preset(zone) : zone;
                out[1] = 0;
            }
            return;
        }
        mask = ((cfg.plugins & KG_PLUGIN_DEV) && devs)
                   ? dev_choose_site(cfg, e, n, zones + rec, devs + rec, pod_view(cfg, e, n, rec, qx), nom, qx, zone) : 0u;
        if (sign == 0) {  // evaluation pass only (a cpuset Reserve runs next)
            if (out && threadIdx.x == 0) out[0] = zone_preset(zone), out[1] = (int32_t)mask, out[2] = nom;
            return;
        }
    }
    __syncthreads();  // every lane has read the state before lane 0 changes it
    if (threadIdx.x != 0) return;
    if (sign < 0 && cpus && allocs && topos) cpuset_release_lane(nodes, zones, allocs, topos, rec, cpus);
    apply_assume(cfg, n, zones + rec, q, zone, sign, split);
    const bool rsv_on = rsv && (cfg.plugins & KG_PLUGIN_RSV) && n[N_RSV_CLASSES] != 0 && e.views;
    if (rsv_on) {
        if (sign > 0) rsv_reserve_dev(e, n, zones + rec, rec, q, nom);
        else rsv_unreserve_dev(e, n, zones + rec, rec, q, rid_in);
    }
    const int32_t rid = sign > 0 ? (nom >= 0 ? (int32_t)e.infos[nom].rid : -1) : rid_in;
    dev_reserve_apply(cfg, e, n, rec, devs ? devs + rec : nullptr, mask, qx, rsv_on ? rid : -1, sign);
    if ((cfg.plugins & KG_PLUGIN_QUOTA) && qx.quota >= 0 && (uint32_t)qx.quota < e.n_quotas) {
        quota_add(e.qstate[qx.quota], q, qx, sign);
        quota_add(e.qstate[e.n_quotas + qx.quota], q, qx, sign);
    }
    if (out) {
        out[0] = zone;
        out[1] = (int32_t)mask;
        out[2] = nom;
        out[3] = nom >= 0 ? (int32_t)e.infos[nom].rid : -1;
    }
}

// launchers

hipError_t launch_ext_replay_step(NodeRec* nodes, ZoneRec* zones, DevRec* devs, const ExtDev& e, const PodsDev& pods,
                                  uint32_t n_pods, uint32_t n_nodes, uint32_t index_base, const KCfg& cfg, bool exact,
                                  const uint32_t* step_base, uint32_t step_off, uint64_t* winners, uint32_t* minors,
                                  uint64_t* buckets, int8_t* zsel, uint32_t* reason, const uint32_t* pos, int32_t* nsel,
                                  RsvStep* rs, uint64_t* rlist, uint32_t* done, const DevClass* dclass, uint32_t n_dclass,
                                  bool fb, uint32_t n0, hipStream_t s) {
    if (n_nodes == 0 || !done) return hipErrorInvalidValue;  // a zero grid would be a malformed dispatch
    if (fb && (exact || reason)) return hipErrorInvalidValue;  // the fast pairs carry no filter bits
    dim3 grid((n_nodes + REPLAY_WG - 1) / REPLAY_WG), block(REPLAY_WG);
#define KG_EXT_REPLAY(EX, F)                                                                                              \
    k_ext_replay<EX, F><<<grid, block, 0, s>>>(nodes, zones, devs, e, pods, n_pods, n_nodes, index_base, cfg, step_base, \
                                               step_off, winners, minors, buckets, zsel, reason, pos, nsel, rs, rlist,   \
                                               done, dclass, n_dclass, n0)
    if (exact) KG_EXT_REPLAY(true, false);
    else if (fb) KG_EXT_REPLAY(false, true);
    else KG_EXT_REPLAY(false, false);
#undef KG_EXT_REPLAY
    return hipGetLastError();
}

hipError_t launch_ext_assume(NodeRec* nodes, ZoneRec* zones, DevRec* devs, const ExtDev& e, const PodsDev& pods,
                             uint32_t pod, uint32_t rec, int32_t zone, uint32_t minors, int64_t sign, const KCfg& cfg,
                             bool exact, int32_t* out, hipStream_t s, int64_t* split, bool rsv, int32_t rid,
                             kg_cpu_alloc* allocs, const kg_cpu_topo* topos, const uint64_t* cpus) {
    if (exact)
        k_ext_assume<true><<<1, 64, 0, s>>>(nodes, zones, devs, e, pods, pod, rec, zone, minors, sign, cfg, out, split, rsv,
                                            rid, allocs, topos, cpus);
    else
        k_ext_assume<false><<<1, 64, 0, s>>>(nodes, zones, devs, e, pods, pod, rec, zone, minors, sign, cfg, out, split, rsv,
                                             rid, allocs, topos, cpus);
    return hipGetLastError();
}

}  // namespace kg
