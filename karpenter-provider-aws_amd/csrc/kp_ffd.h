// kp_ffd.h — the Solve's single-workgroup first-fit-decreasing loop (ffd_solve) and its device helpers, shared by
// the translation units that instantiate it (kp_ffd_*.hip: one group of kernel entry points each, so the
// instantiations compile in parallel) and kp_kernels.hip (launchers, LDS plan).  See kp_kernels.hip for the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "kp_device.h"
#include "kp_eval.h"
#include "kp_gosort.h"
#include "kp_layout.h"

// wave-count namespace (kp_layout.h KP_WNS): the 4-wave topology units and the 8-wave units hold distinct
// definitions of the wave-shaped types (FfdShared, TeamBuf ...) and of every helper that uses them
namespace KP_WNS {

#ifdef KP_NO_TOPO
#define KP_TOPO_ON 0  // A/B builds only (tools/ab_variants.sh): topology code compiled out
#else
#define KP_TOPO_ON 1
#endif

// ExistingNode.Add's requirement merge of class c into node j (wave 0; only solves whose classes carry
// NotIn/DoesNotExist keys).  When node j's requirements change, its XT column is recomputed for every class.
__device__ inline void existing_merge(const KpDev& d, int j, int c, int lane) {
    const int k0 = d.cls_xkoff[c], nk = d.cls_xkoff[c + 1] - k0;
    ReqHdr* nh = d.ex_hdr + (size_t)j * d.K;
    uint64_t* nwp = d.ex_words + (size_t)j * d.DW;
    bool ch = false;
    for (int i = lane; i < nk; i += 64) {
        const int k = d.cls_xkeys[k0 + i];
        ReqHdr A = nh[k];
        ch |= req_merge_inplace(d, k, A, nwp + d.woff[k], d.cls_hdr[(size_t)c * d.K + k],
                                d.cls_words + (size_t)c * d.DW + d.woff[k]);
        nh[k] = A;
    }
    if (!ballot(ch)) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");  // the merged requirements are visible to every lane
    const int w = j >> 6;
    const uint64_t bm = 1ull << (j & 63);
    for (int cc = lane; cc < d.C; cc += 64) {
        const bool ok = d.ex_static[j] && (d.ex_tol[(size_t)cc * d.EW + w] & bm) && node_compatible(d, nh, nwp, cc);
        if (ok) atomicOr((unsigned long long*)&d.XT[(size_t)cc * d.EW + w], (unsigned long long)bm);
        else atomicAnd((unsigned long long*)&d.XT[(size_t)cc * d.EW + w], (unsigned long long)~bm);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------------------------------------
// Solve: single-workgroup first-fit-decreasing
// ------------------------------------------------------------------------------------------------
// Fixed part of the FFD kernel's LDS.  The variable-size tables follow it at the offsets of the LDS plan
// (kp_ffd_plan_lds): slice keys/order and last absorbed class per NodeClaim, the staged allocatable / offering /
// multi-valued label tables, and the quick-accept headroom table hr[lds_A][lds_nq].
struct FfdShared {
    int fastp[2][KP_NWAVES];
    WaveScratch ws[KP_NWAVES];
    TeamBuf team[2];               // topology pods: the block evaluates one candidate at a time (eval_wave TEAM)
    ClassCache CC;
    Roles roles;
    int slot_zone[KP_MAX_SLOTS], slot_ct[KP_MAX_SLOTS], slot_zoneid[KP_MAX_SLOTS];
    int64_t pod_req[KP_MAX_R];
    int cand_pos[2][KP_NWAVES];
    int acc[2][KP_NWAVES];
    int tacc[KP_NWAVES];
    int n_cand[2], scan_done[2], scan_next[2];
    int sstack[64 * 5];
    int bred[2][KP_NWAVES];        // block_sort_move: per-wave first match, double-buffered by round
    int eager, eager_pos, eager_e; // block_sort_move applied [eager_pos, eager_e) ahead of the add() that sorts
    // control state: owned by wave 0 inside its fast loop, by the block between the slow-path barriers
    int N, qhead, qcount, done, cur_pod, cur_cls, cur_shape, prev_shape;
    int dirty_kind, dirty_pos, seq, err, cls_fill, scan_start, any_rej;
    int rej_volatile;              // a candidate of the current pod was rejected for a reason that may not last
                                   // (topology counts): the next pod of the shape rescans from the start
    int rel_flag;                  // a reservation ID's capacity came back from 0 (commit_reservations): the
                                   // reservation-dependent rejections memoised so far may no longer hold
    int epoch;                     // lastLen generation: Queue.Push(pod, relaxed = true) clears lastLen
    int relaxed;                   // a pod relaxed since wave 0 last loaded its queue window (its lastLens are stale)
    uint64_t born;                 // late topology identities created so far (KpDev.tg_late)
    int xstart;                    // every existing node < xstart has rejected the current shape
    uint64_t cur_tol;              // tolerations word of the current shape's class (bit 63: no requirement keys)
    int32_t cur_pq[KP_LDS_AXES];   // scaled quick-accept requests of the current shape
    int64_t shape_req[KP_MAX_R];   // requests of the current shape (pending-total flush)
    long long st[ST_COUNT];
    // topology prefilter of the current pod (topo_prefilter_setup): a NodeClaim whose own requirements admit no
    // domain a constraining group allows cannot accept the pod, and is skipped without an evaluation
    int tp_n, topo_pod, topo_quick;
    int ex_placed;                 // the current topology pod went to this existing node (-1: none accepted it)
    // add() tries the existing nodes before sort.Slice: a topology pod meets a pending slice sort (dirty_kind, eager) with
    // the existing nodes still untried — the block tries them first (topo_defer) and, when none takes the pod, hands it
    // back to wave 0 (topo_resume) for the sort; topo_exdone: the block skips the existing nodes on that pass
    int topo_defer, topo_resume, topo_exdone;
    int tp_all;                    // the prefilter holds every constraining group (at most KP_SNAP_ROWS)
    // the static entries (KpTopoCons) of class tp_cls's first KP_SNAP_ROWS constraining groups and its group count: the
    // setup of the next pod of that class reads them here (set behind the barrier after a setup, read after the next)
    int tp_cls, tp_nall;
    KpTopoCons tp_T[KP_SNAP_ROWS];
    // the recording entries (KpTopoRec) of class tr_cls when it has at most KP_SNAP_ROWS (wave 0's quick-accept Record)
    int tr_cls, tr_n;
    KpTopoRec tr_R[KP_SNAP_ROWS];
    int tp_k[KP_SNAP_ROWS];        // value-keyed group: key; hostname group: -1 - row of tg_hcnt
    int tp_lo[KP_SNAP_ROWS], tp_hi[KP_SNAP_ROWS];  // hostname group: the host's count must lie in [lo, hi]
    int tp_cmp[KP_SNAP_ROWS];      // value-keyed: a complement (NotIn) NodeClaim requirement is not prefiltered
    uint64_t tp_elig[KP_SNAP_ROWS]; // value-keyed: allowed domains ∩ the pod's domains
    TopoSnap* tsnap;               // topology solves: the pod's value-keyed group counts for topo_narrow (dynamic LDS,
                                   // EvalEnv.snap); null otherwise, so other solves keep that LDS for quick-accept rows
};

// Once per pod of a class with constraining topology groups: the per-group conditions topo_narrow applies, reduced to
// what depends on the candidate (its host's count, or its own domains of the key).  Exact up to the NotIn/DoesNotExist
// Compatible exception, which the prefilter leaves to the evaluation.  Group e is set up by wave e: the groups'
// dependent loads overlap instead of queueing on wave 0.  A class constrained by more than KP_SNAP_ROWS groups is
// prefiltered by its first KP_SNAP_ROWS (a superset of the candidates that pass all: evaluations stay exact, read the
// global counters, and the quick accept is off).
__device__ inline void topo_prefilter_setup(const KpDev& d, FfdShared& S, int c, int wave, int lane) {
    const bool hit = S.tp_cls == c;  // the previous setup's class: its static entries are in LDS
    const int t0 = hit ? 0 : d.cls_tcoff[c], nall = hit ? S.tp_nall : d.cls_tcoff[c + 1] - t0;
    const int nt = nall < KP_SNAP_ROWS ? nall : KP_SNAP_ROWS;
    for (int e = wave; e < nt; e += KP_NWAVES) {
        // the entry's static operands (KpTopoCons), then the group's counts: one round of independent loads
        KpTopoCons T = hit ? S.tp_T[e] : d.cls_tce[t0 + e];
        if (!hit && lane == 0) S.tp_T[e] = T;
        if (d.late_sib) {  // a variant group: the identity's born variant (its minDomains)
            T.g = topo_variant(d, T.g, S.born);
            T.mindom = d.tg_info[T.g].w;
        }
        const int g = T.g, type = T.flags & TG_TYPE, self = (T.flags >> 2) & 1;
        int k = T.key, lo = 0, hi = INT32_MAX, cmp = 0;
        uint64_t elig = 0;
        if (T.flags & 8) {  // hostname group: the candidate's host count must lie in [lo, hi]
            if (type == 0) {
                hi = T.skew - self;
            } else if (type == 2) {
                hi = 0;
            } else {
                lo = (self && host_aff_unseeded<false>(d, T, g, nullptr, lane)) ? 0 : 1;
            }
        } else {
            const bool valid = (T.vmask >> lane) & 1ull;
            SnapRow& Z = S.tsnap->r[e];
            const uint64_t known = ld_u64(&d.tg_known[g]);
            const int cnt_raw = ld_i32(&d.tg_cnt[(size_t)g * 64 + lane]);
            const uint8_t rk = d.vrank[(size_t)k * 64 + lane];
            const int cnt = (valid && ((known >> lane) & 1ull)) ? cnt_raw : 0;
            // topo_narrow's view of the group for every candidate of this pod (TopoSnap)
            Z.cnt[lane] = cnt;
            Z.rk[lane] = valid ? rk : 0xFFu;
            if (lane == 0) {
                Z.known = known;
                Z.podhas = T.podhas;
            }
            // the pod's domains: its requirement for the key (every class a value-keyed group constrains carries the key,
            // a topology-only key as Exists)
            const bool pod_has = (T.podhas >> lane) & 1ull;
            const bool kn = valid && ((known >> lane) & 1ull);
            if (type == 0) {
                const uint64_t sup = ballot(kn && pod_has);
                int mn = wave_min_i32((kn && pod_has) ? cnt : INT32_MAX);
                if (T.mindom > 0 && __popcll(sup) < T.mindom) mn = 0;
                elig = ballot(kn && pod_has && (int64_t)cnt + self - (int64_t)mn <= (int64_t)T.skew);
            } else if (type == 2) {
                elig = ballot(kn && cnt == 0 && pod_has);
            } else {
                elig = ballot(kn && cnt > 0 && pod_has);
                cmp = 1;
                if (!elig) {
                    if (self) elig = ballot(kn && pod_has);
                    else cmp = 0;  // no domain at all: Get is empty whatever the node requirement
                }
            }
        }
        if (lane == 0) {
            S.tp_k[e] = k;
            S.tp_lo[e] = lo;
            S.tp_hi[e] = hi;
            S.tp_cmp[e] = cmp;
            S.tp_elig[e] = elig;
        }
    }
    if (wave == 0 && lane == 0) {
        S.tp_n = nt;
        S.tp_all = nall <= KP_SNAP_ROWS;
        S.tp_nall = nall;
    }
}

__device__ __forceinline__ bool topo_prefilter_pass(const KpDev& d, const FfdShared& S, int nc) {
    bool ok = true;
    for (int e = 0; e < S.tp_n && ok; e++) {
        const int k = S.tp_k[e];
        if (k < 0) {
            const int cnt = ld_i32(&d.tg_hcnt[(size_t)(-1 - k) * d.HN + d.E + nc]);
            ok = cnt >= S.tp_lo[e] && cnt <= S.tp_hi[e];
        } else {
            const uint32_t fl = d.nc_hdr[(size_t)nc * d.K + k].flags;
            const uint64_t w = d.nc_words[(size_t)nc * d.DW + d.woff[k]];
            if (!(fl & RF_DEF)) ok = S.tp_elig[e] != 0;
            else if (fl & RF_CMP) ok = S.tp_cmp[e] || (~w & S.tp_elig[e]) != 0;
            else ok = (w & S.tp_elig[e]) != 0;
        }
    }
    return ok;
}

// wave 0: the first slice position in [start, N) that has not rejected the shape, whose template's taints the class
// tolerates (tol: bit j = template j) and that passes the topology prefilter (N if none).  Two 64-position chunks per
// round (KP_TSCAN_U) so the prefilter's global loads of 64 * KP_TSCAN_U NodeClaims overlap.
#ifndef KP_TSCAN_U
#define KP_TSCAN_U 2
#endif
__device__ inline int topo_scan(const KpDev& d, const FfdShared& S, const uint32_t* skey, const uint16_t* sord,
                                const uint8_t* stmpl, uint64_t tol, int N, int start, int lane) {
    constexpr int U = KP_TSCAN_U;
    for (int base = start; base < N; base += 64 * U) {
        bool ok[U];
        int nc[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int p = base + u * 64 + lane;
            ok[u] = p < N && !(skey[p] >> 31);
            nc[u] = ok[u] ? (int)sord[p] : 0;
            ok[u] = ok[u] && ((tol >> stmpl[nc[u]]) & 1ull);
        }
        for (int e = 0; e < S.tp_n; e++) {
            const int k = S.tp_k[e];
            if (k < 0) {
                const int32_t* row = d.tg_hcnt + (size_t)(-1 - k) * d.HN + d.E;
                const int lo = S.tp_lo[e], hi = S.tp_hi[e];
                int cnt[U];
#pragma unroll
                for (int u = 0; u < U; u++) cnt[u] = ok[u] ? ld_i32(row + nc[u]) : 0;
#pragma unroll
                for (int u = 0; u < U; u++) ok[u] = ok[u] && cnt[u] >= lo && cnt[u] <= hi;
            } else {
                const uint64_t el = S.tp_elig[e];
                const bool cmp = S.tp_cmp[e];
                uint32_t fl[U];
                uint64_t w[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    fl[u] = ok[u] ? d.nc_hdr[(size_t)nc[u] * d.K + k].flags : 0u;
                    w[u] = ok[u] ? d.nc_words[(size_t)nc[u] * d.DW + d.woff[k]] : 0ull;
                }
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const bool pass = !(fl[u] & RF_DEF) ? el != 0 : (fl[u] & RF_CMP) ? (cmp || (~w[u] & el) != 0)
                                                                                       : (w[u] & el) != 0;
                    ok[u] = ok[u] && pass;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t m = ballot(ok[u]);
            if (m) return base + u * 64 + __ffsll((unsigned long long)m) - 1;
        }
    }
    return N;
}

// The whole block: the first slice position in [start, N) that passes topo_scan's tests (N if none).  Wave w scans the
// SPAN = 64 * KP_TSCAN_U positions [base + SPAN w, base + SPAN (w + 1)) of each round (one barrier per round), and the
// round's lowest survivor wins; rounds stop at the first that has one.  red: [2][KP_NWAVES] LDS, by round parity.
__device__ inline int topo_scan_block(const KpDev& d, const FfdShared& S, const uint32_t* skey, const uint16_t* sord,
                                      const uint8_t* stmpl, uint64_t tol, int N, int start, int (*red)[KP_NWAVES],
                                      int wave, int lane) {
    constexpr int SPAN = 64 * KP_TSCAN_U;
    for (int base = start, r = 0; base < N; base += SPAN * KP_NWAVES, r ^= 1) {
        const int wb = base + SPAN * wave, we = wb + SPAN < N ? wb + SPAN : N;
        int f = wb < N ? topo_scan(d, S, skey, sord, stmpl, tol, we, wb, lane) : N;
        if (f >= we) f = N;  // topo_scan reports "none" as its end bound
        if (lane == 0) red[r][wave] = f;
        __syncthreads();
        int m = N;
        for (int w = 0; w < KP_NWAVES; w++) m = red[r][w] < m ? red[r][w] : m;
        if (m < N) return m;
    }
    return N;
}

// Every value-keyed group of the pod already sees a single domain on NodeClaim nc (its requirement for the key is
// In [one value]), so AddRequirements cannot narrow it (the prefilter has admitted that value).  Lane e reads group e's
// key of the NodeClaim's digest (one round of loads).
__device__ inline bool topo_pinned(const KpDev& d, const FfdShared& S, int nc, int lane) {
    bool ok = true;
    if (lane < S.tp_n) {
        const int k = S.tp_k[lane];
        if (k >= 0) {
            const uint32_t fl = d.nc_hdr[(size_t)nc * d.K + k].flags;
            const uint64_t w = d.nc_words[(size_t)nc * d.DW + d.woff[k]];
            ok = (fl & RF_DEF) && !(fl & RF_CMP) && __popcll(w) == 1;
        }
    }
    return ballot(!ok) == 0;
}

// The requirement merge of NodeClaim.Add(pod of class c) on NodeClaim nc is a no-op: for every key the class constrains
// (keys carried only for topology narrowing aside), the NodeClaim has the key and Requirement.Intersection leaves it as it
// is (header and values), and the pair passes Compatible.  Then the Add keeps the NodeClaim's requirements, so its options
// stay compatible and its offerings the same: the topology quick accept applies as for a NodeClaim that absorbed the
// class (wave 0; ws.words is free scratch here).
__device__ inline bool merge_noop(const KpDev& d, FfdShared& S, int nc, int c, int lane) {
    const ReqHdr* h = d.nc_hdr + (size_t)nc * d.K;
    const uint64_t* w = d.nc_words + (size_t)nc * d.DW;
    return S.CC.cls == c ? merge_noop_cc(d, S.CC, S.ws[0], h, w, lane) : merge_noop_at(d, S.ws[0], h, w, c, lane);
}

// Topology.Record of a quick accept onto NodeClaim nc (template tmpl): its requirements are unchanged by the Add, so
// every recorded domain comes from its digest (hostname groups: its host E + nc).  CF_TOPO_QREC guarantees that no
// recording group needs the node-affinity filter of another class.  Lane i takes recording entry i (KpTopoRec) and its
// key of the NodeClaim's digest, so the entries' loads form one round; the counts are then added entry by entry.
__device__ inline void topo_record_quick(const KpDev& d, FfdShared& S, int c, int nc, int tmpl, uint64_t born, int lane) {
    const bool hit = S.tr_cls == c;  // the entries are in LDS (wave 0 alone reads and writes them)
    const int r0 = hit ? 0 : d.cls_troff[c], nr = hit ? S.tr_n : d.cls_troff[c + 1] - r0;
    const bool keep = !hit && nr <= KP_SNAP_ROWS;
    for (int base = 0; base < nr; base += 64) {
        const int i = base + lane;
        KpTopoRec R{};
        uint32_t fl = 0;
        uint64_t w = 0;
        bool live = false;
        if (i < nr) {
            R = hit ? S.tr_R[i] : d.cls_tre[r0 + i];
            if (keep) S.tr_R[i] = R;
            live = !((R.skip >> tmpl) & 1ull) && (R.late < 0 || ((born >> R.late) & 1ull));
            if (live && !(R.flags & 8)) {
                fl = d.nc_hdr[(size_t)nc * d.K + R.key].flags;
                w = d.nc_words[(size_t)nc * d.DW + d.woff[R.key]];
                const int type = R.flags & TG_TYPE;
                const bool inv = (R.flags >> 2) & 1;
                // Get() of an undefined key is Exists (no values); spread / affinity record a single value only
                live = (fl & RF_DEF) && !(!inv && type != 2 && ((fl & RF_CMP) || __popcll(w) != 1));
            }
        }
        for (uint64_t m = ballot(live); m; m &= m - 1) {
            const int j = __ffsll((unsigned long long)m) - 1;
            const int g = rl32(R.g, j), flags = rl32(R.flags, j), key = rl32(R.key, j);
            if (flags & 8) {
                if (lane == 0) {
                    const int old = atomicAdd(&d.tg_hcnt[(size_t)(-1 - key) * d.HN + d.E + nc], 1);
                    if (old == 0) atomicAdd(&d.tg_pos[g], 1);
                }
                continue;
            }
            const uint64_t wv = rl64(w, j);
            if ((wv >> lane) & 1ull) atomicAdd(&d.tg_cnt[(size_t)g * 64 + lane], 1);
            if (lane == 0 && wv) atomicOr((unsigned long long*)&d.tg_known[g], (unsigned long long)wv);
        }
    }
    if (keep && lane == 0) {
        S.tr_n = nr;
        S.tr_cls = c;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// wave 0: collect up to KP_NWAVES slice positions >= start whose NodeClaim has not rejected the current shape, whose
// template's taints the pod's class tolerates (NodeClaim.Add's first test; tol bit j = template j) and that passes the
// topology prefilter of the current pod
__device__ inline void collect_candidates(const KpDev& d, FfdShared& S, const uint32_t* key, const uint16_t* ord,
                                          const uint8_t* stmpl, uint64_t tol, int N, int start, int buf, int lane) {
    int cnt = 0, pos = start, next = N;
    // topology pods: at most d.topo_cands candidates per round (the first prefilter survivor usually accepts; fewer waves
    // evaluating leaves each its own SIMD)
    const int L = S.tp_n ? d.topo_cands : KP_NWAVES;
    while (pos < N) {
        const int p = pos + lane;
        bool c = p < N && !(key[p] >> 31);
        if (c) c = (tol >> stmpl[ord[p]]) & 1ull;
        if (S.tp_n && c) c = topo_prefilter_pass(d, S, ord[p]);
        const uint64_t m0 = __ballot(c);
        if (S.tp_n && m0 && cnt + __popcll(m0) < L) {
            // topology pods: the first prefilter survivor usually accepts; end the round with this window rather than
            // paying the prefilter's loads for up to 8 candidates (the next round continues after it)
            const int rank = cnt + __popcll(m0 & ((1ull << lane) - 1ull));
            if (c) S.cand_pos[buf][rank] = p;
            cnt += __popcll(m0);
            pos += 64;
            if (lane == 0) {
                S.n_cand[buf] = cnt;
                S.scan_next[buf] = pos < N ? pos : N;
                S.scan_done[buf] = pos >= N;
            }
            return;
        }
        const uint64_t m = __ballot(c);
        const int rank = cnt + __popcll(m & ((1ull << lane) - 1ull));
        if (c && rank < L) S.cand_pos[buf][rank] = p;
        const int tot = cnt + __popcll(m);
        if (tot >= L) {
            const uint64_t last = __ballot(c && rank == L - 1);
            next = pos + __ffsll((unsigned long long)last);  // position after the last collected candidate
            cnt = L;
            break;
        }
        cnt = tot;
        pos += 64;
    }
    if (lane == 0) {
        S.n_cand[buf] = cnt;
        S.scan_next[buf] = cnt == L ? next : N;
        S.scan_done[buf] = (cnt < L) || next >= N;
    }
}

// types whose Capacity exceeds a NodePool's remaining limits (filterByRemainingResources)
// Types of template j whose capacity fits its NodePool's remaining limits (the NewNodeClaim limit filter): tmpl_lmask
// holds them by word (lane w: word w), set at kernel start and recomputed for a template when a NodeClaim of it takes
// capacity off its limits (limit_mask_update), so a template evaluation reads one word per lane.
__device__ __forceinline__ uint64_t limit_filter(const KpDev& d, int j, uint64_t o, int lane) {
    return lane < d.TW ? o & d.tmpl_lmask[(size_t)j * d.TW + lane] : o;
}

// tmpl_lmask[j][w] from the current remaining limits (one wave; every limited axis of j: capacity <= remaining).
__device__ inline void limit_mask_update(const KpDev& d, int j, int lane) {
    uint32_t lm = 0;
    for (int r = 0; r < d.R; r++)
        if (d.limit_set[(size_t)j * d.R + r]) lm |= 1u << r;
    uint64_t mine = ~0ull;
    for (int w = 0; w < d.TW && lm; w++) {
        const int t = w * 64 + lane;
        bool keep = t < d.T;
        for (uint32_t m = lm; m && keep; m &= m - 1) {
            const int r = __ffs(m) - 1;
            keep = d.cap[(size_t)r * d.T + t] <= ld_req(&d.remaining[(size_t)j * d.R + r]);
        }
        const uint64_t nb = ballot(keep);
        if (lane == w) mine = nb;
    }
    if (lane < d.TW) d.tmpl_lmask[(size_t)j * d.TW + lane] = mine;
}

__device__ __forceinline__ long long prof_clock(const KpDev& d) { return d.profile ? __builtin_amdgcn_s_memtime() : 0; }


// The winner's reservations (one wave; lane r: word r of the held set): ReservationManager.Reserve for the
// reservations newly held, Release for those the Add no longer holds (NodeClaim.Add's reservedOfferings update), then
// the NodeClaim's held set and liveness.  fresh: a NodeClaim being created (it held nothing).
__device__ __forceinline__ void commit_reservations(const KpDev& d, int32_t* rcap, const WaveScratch& ws, int nc,
                                                    bool fresh, int* rel_flag, int lane) {
    const int RW = d.ro_ridw;
    if (lane < RW) {
        uint64_t* hp = d.nc_held + (size_t)nc * RW + lane;
        const uint64_t old = fresh ? 0ull : ld_u64(hp), nh = ws.minbits[lane];
        for (uint64_t x = nh & ~old; x; x &= x - 1) rcap[lane * 64 + __ffsll((unsigned long long)x) - 1]--;
        for (uint64_t x = old & ~nh; x; x &= x - 1)
            if (rcap[lane * 64 + __ffsll((unsigned long long)x) - 1]++ == 0) *rel_flag = 1;
        __hip_atomic_store(hp, nh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) __hip_atomic_store(&d.nc_rlive[nc], ws.rlive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// lane r: word r of the reservations NodeClaim nc holds
__device__ __forceinline__ uint64_t held_word(const KpDev& d, int nc, int lane) {
    return lane < d.ro_ridw ? ld_u64(&d.nc_held[(size_t)nc * d.ro_ridw + lane]) : 0ull;
}

// Scheduler.Solve.  Wave 0 runs the queue, the sort.Slice emulation and the first-fit scan for as many pods as it
// can resolve alone: a pod whose first non-rejected NodeClaim (slice order) has already absorbed the pod's class
// and whose witness type still fits is placed without an evaluation (exact: see pick_witness).  Any other pod is
// handed to all 8 waves (the slow path: NodeClaim.Add of up to 8 candidates at once, or the templates).
// ExistingNode.Add over the existing nodes for a pod of a topology class (wave 0; DESIGN.md §4 "Topology over a
// cluster"): the first node in scheduling order that is tolerated, Compatible, has headroom and passes
// Topology.AddRequirements takes the pod; its requirements, the domain counts and its headroom are updated.  Kept out
// of line: it runs only for clusters, and inlined it would weigh on the topology instantiations' register plan.
static __device__ __attribute__((noinline)) int existing_topo_scan(const KpDev* __restrict__ dp, FfdShared& S, int pod, int lane) {
    const KpDev& d = *dp;
    const int K = d.K;
    const int c = S.cur_cls;
    const bool cons = (d.cls_flags[c] & CF_TOPO_CONS) != 0;
    int placed = -1;
    for (int base = 0; base < d.E && placed < 0; base += 64) {
        const int j = base + lane;
        bool cand = false;
        if (j < d.E) {
            const uint64_t xw = __hip_atomic_load(&d.XT[(size_t)c * d.EW + (j >> 6)], __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
            cand = (xw >> (j & 63)) & 1ull;
            for (int ai = 0; ai < d.n_active && cand; ai++)
                cand = S.pod_req[d.active_axes[ai]] <= ld_req(&d.ex_head[(size_t)ai * d.E + j]);
        }
        uint64_t m = ballot(cand);
        while (m) {
            const int jj = base + __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            const bool ok = cons ? existing_topo_try<true>(d, S.CC, S.ws[0], jj, lane)
                                 : existing_topo_try<false>(d, S.CC, S.ws[0], jj, lane);
            if (ok) {
                placed = jj;
                break;
            }
        }
    }
    if (placed >= 0) {
        existing_topo_commit(d, S.CC, S.ws[0], placed, lane);
        topo_record(d, S.CC, S.ws[0], d.ex_hdr + (size_t)placed * K, d.ex_words + (size_t)placed * d.DW,
                    placed, 0, false, lane, placed, nullptr, S.born);
        if (lane < d.n_active) {
            const int64_t x = S.pod_req[d.active_axes[lane]];
            if (x) atomicAdd((unsigned long long*)&d.ex_head[(size_t)lane * d.E + placed], (unsigned long long)(-x));
        }
        if (lane == 0) {
            d.pod_result[pod] = -2 - placed;
            d.pod_order[pod] = S.seq++;
            S.scan_start = 0;
            S.st[ST_EXIST_PLACED] += 1;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    return placed;
}

// PREF: the solve relaxes preferences or runs MIN_VALUES_POLICY=BestEffort; false compiles that code out, so the
// common instantiations keep the register plan they had without it.
// HBM: the slice arrays (9 B per in-flight NodeClaim) live in HBM (d.g_key ...) because the solve is planned for more
// NodeClaims than LDS holds beside the fixed tables (kp_ffd_plan_lds sets d.slice_hbm); other instantiations keep them
// in LDS and address them with ds instructions.
// The slow path's commit leaves one slice change for sort.Slice at the next add(): position pos gained a pod.  When
// pdqsort's handling of it is the stable move (sort_slice_after_change: no inversion, or n <= 12, or n >= 50 and pos
// is not a pivot sample) the whole block applies it here, 512 positions per step, instead of wave 0 alone at its
// next pop; otherwise the change stays for wave 0.  Every thread calls it (uniform control, barriers inside).
__device__ inline void block_sort_move(FfdShared& S, SortSlice sl, int tid, int nthr) {
    const int n = S.N, pos = S.dirty_pos;
    if (S.dirty_kind != 1 || pos + 1 >= n) return;
    const uint32_t kr = sl.key[pos], kv = kr & KEYMASK;
    if ((sl.key[pos + 1] & KEYMASK) < kv) {
        if (!(n <= 12 || (n >= 50 && !is_pivot_sample(n, pos)))) return;  // wave 0: pivot hint or pdqsort
        const int lane = tid & 63, wave = tid >> 6;
        // run end: the first position after pos whose key is >= the new key
        int e = n;
        for (int base = pos + 1, r = 0; base < n; base += nthr, r ^= 1) {
            const int p = base + tid;
            const uint64_t m = __ballot(p < n && (sl.key[p] & KEYMASK) >= kv);
            if (lane == 0) S.bred[r][wave] = m ? base + wave * 64 + __ffsll((unsigned long long)m) - 1 : n;
            __syncthreads();
            for (int w = 0; w < KP_NWAVES; w++) e = S.bred[r][w] < e ? S.bred[r][w] : e;
            if (e < n) break;
        }
        // [pos, e): element pos moves to e - 1, the rest shift left by one, 512 positions per step in order
        const uint16_t fo = sl.ord[pos];
        for (int base = pos; base < e - 1; base += nthr) {
            const int i = base + tid;
            uint16_t o = 0;
            uint32_t k = 0;
            if (i < e - 1) {
                o = sl.ord[i + 1];
                k = sl.key[i + 1];
            }
            __syncthreads();
            if (i < e - 1) {
                sl.ord[i] = o;
                sl.key[i] = k;
            }
            __syncthreads();
        }
        if (tid == 0) {
            sl.ord[e - 1] = fo;
            sl.key[e - 1] = kr;
            // Go sorts at the next add() that reaches the NodeClaims: if none does, the move is undone at the end
            S.eager = 1;
            S.eager_pos = pos;
            S.eager_e = e;
        }
    }
    __syncthreads();  // every thread has read dirty_kind
    if (tid == 0) S.dirty_kind = 0;
}

#ifndef KP_TOPO_BLOCK_SCAN
#define KP_TOPO_BLOCK_SCAN 1  // A/B builds: 0 = topology prefilter setup and scan on wave 0 alone (round 4)
#endif
#ifndef KP_TEAM_FIRST_RESV
#define KP_TEAM_FIRST_RESV 0  // 0: no block-evaluated first candidate in the RESV instantiations (its registers cost config 5 15 %)
#endif
#ifndef KP_TEAM_FIRST_TOPO
#define KP_TEAM_FIRST_TOPO 1  // A/B builds: 0 compiles the block-evaluated first candidate out of the TOPO instantiations
#endif
#ifndef KP_TEAM_TMPL
#define KP_TEAM_TMPL 1         // the templates evaluated one at a time by the whole block (the instantiations without
                              // reserved offerings or topology groups: config 2 91.9 -> 90.5 ms; config 3 unchanged)
#endif
#ifndef KP_TEAM_TMPL_RESV
#define KP_TEAM_TMPL_RESV 0    // A/B builds: 1 also in the RESV instantiations
#endif
#ifndef KP_NOOP_RESV
#define KP_NOOP_RESV 1        // A/B builds: 0 compiles the no-op merge quick accept out of the RESV instantiations
#endif
template <bool RESV, bool TOPO, bool PREF, bool HBM = false>
__device__ __forceinline__ void ffd_solve(KpDev d) {
    constexpr bool TOPO_ON = KP_TOPO_ON && TOPO;  // the solve has topology groups
    extern __shared__ __attribute__((aligned(16))) char smem[];
    FfdShared& S = *reinterpret_cast<FfdShared*>(smem);
    uint32_t* const skey = HBM ? d.g_key : reinterpret_cast<uint32_t*>(smem + d.off_key);    // len(Pods) by slice position
    uint16_t* const sord = HBM ? d.g_ord : reinterpret_cast<uint16_t*>(smem + d.off_ord);    // NodeClaim id by slice position
    uint16_t* const slast = HBM ? d.g_last : reinterpret_cast<uint16_t*>(smem + d.off_last); // last absorbed class by NodeClaim id
    uint8_t* const stmpl = HBM ? d.g_tmpl : reinterpret_cast<uint8_t*>(smem + d.off_tmpl);   // template by NodeClaim id
    int64_t* const sAlloc = reinterpret_cast<int64_t*>(smem + d.off_alloc);
    uint64_t* const sAvail = reinterpret_cast<uint64_t*>(smem + d.off_avail);
    uint16_t* const sMulti = reinterpret_cast<uint16_t*>(smem + d.off_multi);
    int32_t* const shr = reinterpret_cast<int32_t*>(smem + d.off_hr);       // [A][NQ] witness headroom
    int64_t* const qw_req = reinterpret_cast<int64_t*>(smem + d.off_qw);    // [64][R] requests of the queue window's pods
    // reserved offerings and the ReservationManager's capacities (RESV instantiation: the catalog has reserved offerings)
    ResvTab* const sRo = RESV ? reinterpret_cast<ResvTab*>(smem + d.off_ro) : nullptr;
    int32_t* const sRcap = RESV ? reinterpret_cast<int32_t*>(smem + d.off_ro + sizeof(ResvTab)) : nullptr;  // [nrid]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nthr = blockDim.x;
    const int T = d.T, TW = d.TW, K = d.K, R = d.R, P = d.P;
    const int TP = d.lds_tpad, NQ = d.lds_nq, A = d.lds_A, NCMAX = d.lds_ncmax;
    // ---- stage the type tables in LDS ----
    for (int i = tid; i < (d.alloc_global ? 0 : d.lds_nstage * TP); i += nthr) {
        const int ai = i / TP, t = i % TP;
        sAlloc[i] = t < T ? d.alloc[(size_t)act_axis(d, ai) * T + t] : 0;
    }
    for (int t = tid; t < TP; t += nthr) sAvail[t] = t < T ? d.avail_zc[t] : 0;
    if (d.multi16)
        for (int i = tid; i < d.n_multi * TP; i += nthr) {
            const int m = i / TP, t = i % TP;
            sMulti[i] = t < T ? d.multi16[(size_t)m * T + t] : 0;
        }
    for (int s = tid; s < KP_MAX_SLOTS; s += nthr) {
        S.slot_zone[s] = s < d.n_slots ? d.slot_zone[s] : 0;
        S.slot_ct[s] = s < d.n_slots ? d.slot_ct[s] : 0;
        S.slot_zoneid[s] = s < d.n_slots ? d.slot_zoneid[s] : -1;
    }
    if (tid < 5) {
        const int rk = tid == 0 ? d.key_zone : tid == 1 ? d.key_ct : tid == 2 ? d.key_zoneid : tid == 3 ? d.key_resvid : d.key_resvtype;
        S.roles.key[tid] = rk;
        S.roles.woff[tid] = rk >= 0 ? d.woff[rk] : 0;
        S.roles.nw[tid] = rk >= 0 ? d.nw[rk] : 0;
    }
    if (RESV) {
        // the ReservationManager (NewReservationManager: every reservation's capacity) and the ResvTab header in LDS;
        // small tables (d.ro_stage) also get their rows staged after the capacities, the header pointing at them
        for (int i = tid; i < d.ro_nrid; i += nthr) sRcap[i] = d.rcap0[i];
        const ResvTab& G = *d.ro;
        const int n = d.ro_n;
        int32_t* st = sRcap + ((d.ro_nrid + 1) & ~1);
        if (d.ro_stage) {
            for (int i = tid; i < n; i += nthr) {
                st[i] = G.type[i];
                st[n + i] = G.zone[i];
                st[2 * n + i] = G.zid[i];
                st[3 * n + i] = G.rid[i];
                st[4 * n + i] = G.ridv[i];
                st[5 * n + i] = G.rtype[i];
            }
            uint64_t* av = reinterpret_cast<uint64_t*>(st + 6 * ((n + 1) & ~1));
            for (int i = tid; i < d.ro_w; i += nthr) av[i] = G.avail[i];
        }
        if (tid == 0) {
            ResvTab h = G;
            if (d.ro_stage) {
                h.type = st;
                h.zone = st + n;
                h.zid = st + 2 * n;
                h.rid = st + 3 * n;
                h.ridv = st + 4 * n;
                h.rtype = st + 5 * n;
                h.avail = reinterpret_cast<const uint64_t*>(st + 6 * ((n + 1) & ~1));
            }
            *sRo = h;
        }
    }
    for (int p = tid; p < P; p += nthr) {
        d.qbuf[p] = d.queue0[p];
        d.last_len[p] = 0;
        d.pod_result[p] = -1;
        d.pod_order[p] = -1;
    }
    for (int j = wave; j < d.NT; j += KP_NWAVES) limit_mask_update(d, j, lane);  // the NodePools' limits of this solve
    int tjoins = 0;  // TEAM evaluations whose join this wave passed (block-uniform): the TeamBuf parity
    if (PREF && d.relax_next)  // a previous execute may have relaxed pods: every pod starts from its input class
        for (int p = tid; p < P; p += nthr) {
            d.pod_cls[p] = d.pod_cls0[p];
            d.pod_shape[p] = d.pod_shape0[p];
            d.last_ep[p] = -1;
        }
    if (tid == 0) {
        S.N = 0;
        S.tp_n = 0;
        S.tp_cls = -1;
        S.tr_cls = -1;
        S.tsnap = d.G > 0 ? reinterpret_cast<TopoSnap*>(smem + d.off_tsnap) : nullptr;
        S.topo_pod = 0;
        S.topo_quick = 0;
        S.topo_defer = 0;
        S.topo_resume = 0;
        S.topo_exdone = 0;
        S.qhead = 0;
        S.qcount = P;
        S.done = 0;
        S.prev_shape = -1;
        S.eager = 0;
        S.dirty_kind = 0;
        S.dirty_pos = 0;
        S.scan_start = 0;
        S.any_rej = 0;
        S.rej_volatile = 0;
        S.rel_flag = 0;
        S.epoch = 0;
        S.relaxed = 0;
        S.born = d.born0;
        S.xstart = 0;
        S.seq = 0;
        S.err = 0;
        S.CC.cls = -1;
        S.cur_cls = -1;
        S.cur_tol = 0;
        for (int i = 0; i < KP_LDS_AXES; i++) S.cur_pq[i] = 0;
        for (int i = 0; i < KP_MAX_R; i++) S.shape_req[i] = 0;
        for (int i = 0; i < ST_COUNT; i++) S.st[i] = 0;
    }
    __syncthreads();
    EvalEnv E;
    E.pt = nullptr;
    E.snap = d.G > 0 ? reinterpret_cast<TopoSnap*>(smem + d.off_tsnap) : nullptr;  // filled per pod by topo_prefilter_setup
    E.alloc = d.alloc_global ? d.alloc_act : sAlloc;
    E.astride = TP;
    E.avail = sAvail;
    E.multi16 = d.multi16 ? sMulti : nullptr;
    E.slot_zone = S.slot_zone;
    E.slot_ct = S.slot_ct;
    E.slot_zoneid = S.slot_zoneid;
    E.roles = &S.roles;
    E.ro = sRo;
    E.type_ro = d.type_ro;
    E.rcap = sRcap;
    E.resv_on = RESV ? d.resv_on : 0;  // provisioning: ReservedOfferingModeStrict (eval_wave's STRICT default)
    {
        uint64_t mmask = 0;
        for (int j = 0; j < d.NT; j++)
            if (d.min_keys[(size_t)j * KP_MAX_CLASS_KEYS] >= 0) mmask |= 1ull << j;
        E.min_tmpl_mask = mmask;
    }
    SortSlice sl{skey, sord};
    // per-lane quick-accept axis (lane a < A) and its scale
    int my_axis = 0, my_shift = 0;
#pragma unroll
    for (int ai = 0; ai < KP_LDS_AXES; ai++)
        if (lane == ai) {
            my_axis = d.active_axes[ai];
            my_shift = d.qshift[ai];
        }
    const long long pop_bound = (long long)P * 64 + 4096;  // Go's loop ends within P·(retries+1) pops
    // wave 0 state that lives across slow-path episodes:
    //   queue window — lane i holds the i-th next queued pod (refilled every 64 pops; pushes land after it):
    //     pod, class, shape, lastLen, tolerations word (bit 31: class has no requirement keys), and
    //     vq[a] = ceil(request[axis a] >> qshift[a]) for the quick-accept axes (clamped to int32).
    int qw_n = 0, qw_used = 0;
    int vp = 0, vc = 0, vshape = 0, vlast = 0;
    uint64_t vtol = 0;
    int32_t vq[KP_LDS_AXES];
#pragma unroll
    for (int ai = 0; ai < KP_LDS_AXES; ai++) vq[ai] = 0;

    for (;;) {
        const long long c_top = (d.profile && tid == 0) ? __builtin_amdgcn_s_memtime() : 0;
        // ================= wave 0: the fast loop =================
        if (wave == 0) {
            const long long c_in = prof_clock(d);
            const int N = S.N;
            int qhead = S.qhead, qcount = S.qcount;
            int seq = S.seq, prev_shape = S.prev_shape, dkind = S.dirty_kind, dpos = S.dirty_pos;
            int sstart = S.scan_start;  // every slice position < sstart has rejected the current shape
            int eager = S.eager;        // a block_sort_move not yet reached by an add() that sorts
            int any_rej = S.any_rej;
            const int ep = S.epoch;
            if (PREF && d.relax_next && S.relaxed) {
                vlast = -1;  // Queue.Push(pod, relaxed): every lastLen read into the window is gone
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                if (lane == 0) S.relaxed = 0;
            }
            if (RESV && S.rel_flag) {
                // a reservation capacity came back from 0: forget the shape's memoised rejections (a reservation-
                // dependent one may now succeed; the others are re-derived on the next scan)
                for (int i = lane; i < N; i += 64) skey[i] &= KEYMASK;
                any_rej = 0;
                sstart = 0;
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                if (lane == 0) S.rel_flag = 0;
            }
            int xstart = S.xstart;
            long long nexist = 0;
            // pods of the current shape placed on existing node xj whose headroom update is still pending (flushed
            // when xj changes; xj is never scanned again within the shape: positions < xstart are skipped)
            int xj = -1, xcnt = 0;
            auto ex_flush = [&]() {
                if (xj >= 0 && xcnt && lane < d.n_active) {
                    int r = 0;
#pragma unroll
                    for (int ai = 0; ai < KP_MAX_R; ai++)
                        if (ai == lane) r = d.active_axes[ai];
                    const int64_t x = S.shape_req[r];
                    if (x) atomicAdd((unsigned long long*)&d.ex_head[(size_t)lane * d.E + xj], (unsigned long long)(-x * xcnt));
                }
                xj = -1;
                xcnt = 0;
            };
            int done = 0, err = S.err;
            int c = S.cur_cls;
            // the current shape's class carries topology (CF_TOPO): such pods are handled by the block
            bool ctopo = TOPO_ON && c >= 0 && (d.cls_flags[c] & CF_TOPO);
            uint64_t tl = S.cur_tol;
            int pq[KP_LDS_AXES];
#pragma unroll
            for (int ai = 0; ai < KP_LDS_AXES; ai++) pq[ai] = S.cur_pq[ai];
            long long popped = S.st[ST_POPPED], scanned = 0, nquick = 0, sfast = 0, sfull = 0, csort = 0, csfull = 0;
            long long cqpop = 0, cqscan = 0, cqcheck = 0, cqcommit = 0;
            long long n_noinv = 0, n_winmove = 0, n_ldssort = 0, n_pivot = 0, n_winload = 0, n_flush = 0, n_shape = 0;
            long long n_r2 = 0, n_rwb = 0, n_rout = 0, n_batch = 0;

            // ---- slice window: lane i mirrors slice position wb + i and its NodeClaim (authoritative while valid) ----
            int wb = -1;
            uint32_t wk = 0xFFFFFFFFu, wo = 0, wm = 0xFFFFu;  // key|rejected, NodeClaim id, lastClass | template << 16
            int32_t wh[KP_LDS_AXES];                            // witness headroom (scaled), -1: never quick
            bool wa = false;                                    // the NodeClaim has absorbed the current class
            int wcnt = 0;                                       // current-shape pods placed since the last flush
#pragma unroll
            for (int ai = 0; ai < KP_LDS_AXES; ai++) wh[ai] = -1;
            auto absorbed = [&](uint32_t m) -> bool {
                return (int)(m & 0xFFFFu) == c || ((tl >> 63) && ((tl >> (m >> 16)) & 1ull));
            };
            // write the window back to LDS and the pending request totals to HBM (same-shape requests are identical)
            auto win_flush = [&]() {
                if (wb < 0) return;
                n_flush++;
                const int q = wb + lane;
                if (q < N) {
                    skey[q] = wk;
                    sord[q] = (uint16_t)wo;
                    if ((int)wo < NQ)
                        for (int ai = 0; ai < A; ai++) shr[ai * NQ + wo] = wh[ai];
                    if (wcnt)
                        for (int r = 0; r < R; r++) {
                            const int64_t x = S.shape_req[r];
                            if (x) atomicAdd((unsigned long long*)&d.nc_req[(size_t)wo * R + r], (unsigned long long)(x * wcnt));
                        }
                }
                wcnt = 0;
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            };
            auto win_load = [&](int base) {
                n_winload++;
                wb = base;
                const int q = wb + lane;
                if (q < N) {
                    wk = skey[q];
                    wo = sord[q];
                    wm = (uint32_t)slast[wo] | ((uint32_t)stmpl[wo] << 16);
#pragma unroll
                    for (int ai = 0; ai < KP_LDS_AXES; ai++) wh[ai] = (ai < A && (int)wo < NQ) ? shr[ai * NQ + wo] : -1;
                } else {
                    wk = 0xFFFFFFFFu;
                    wo = 0;
                    wm = 0xFFFFu;
#pragma unroll
                    for (int ai = 0; ai < KP_LDS_AXES; ai++) wh[ai] = -1;
                }
                wa = q < N && absorbed(wm);
                wcnt = 0;
            };
            int resume = TOPO_ON ? S.topo_resume : 0;  // the current pod comes back from the block for the sort
            for (;;) {
              int p, off, shape;
              long long t_a;
              if (TOPO_ON && resume) {
                resume = 0;
                p = S.cur_pod;
                off = -1;
                shape = prev_shape;
                t_a = prof_clock(d);
              } else {
                if (qcount == 0 || err) {
                    done = 1;
                    break;
                }
                if (popped > pop_bound) {  // a runaway loop is reported, not hung
                    err = 2;
                    done = 1;
                    break;
                }
                // Queue.Pop through a register window over the next <= 64 queue slots (pushes never land inside)
                if (qw_used >= qw_n) {
                    const int wn = qcount < 64 ? qcount : 64;
                    if (lane < wn) {
                        int pos = qhead + lane;
                        if (pos >= P) pos -= P;
                        vp = d.qbuf[pos];
                        vc = d.pod_cls[vp];
                        vshape = d.pod_shape[vp];
                        vlast = (PREF && d.last_ep && d.last_ep[vp] != ep) ? -1 : d.last_len[vp];
                        vtol = (d.tol[vc] & ~(1ull << 63)) | ((d.cls_flags[vc] & 4u) ? (1ull << 63) : 0ull);
                        for (int r = 0; r < R; r++) qw_req[lane * R + r] = d.pod_req[(size_t)vp * R + r];
#pragma unroll
                        for (int ai = 0; ai < KP_LDS_AXES; ai++) {
                            const int64_t pr = ai < A ? d.pod_req[(size_t)vp * R + d.active_axes[ai]] : 0;
                            const int64_t x = (pr + ((1ll << d.qshift[ai]) - 1)) >> d.qshift[ai];
                            vq[ai] = x > 0x7FFFFFFF ? 0x7FFFFFFF : (int32_t)x;
                        }
                    }
                    qw_n = wn;
                    qw_used = 0;
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                }
                t_a = prof_clock(d);
                off = qw_used;
                if (rl32(vlast, off) == qcount) {
                    done = 1;
                    break;
                }
                p = rl32(vp, off);
                shape = rl32(vshape, off);
                qw_used++;
                qhead = qhead + 1 == P ? 0 : qhead + 1;
                qcount--;
                popped++;
                if (shape != prev_shape) {
                    n_shape++;
                    ex_flush();
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nodes are scanned again from 0
                    xstart = 0;
                    win_flush();  // pending totals belong to the previous shape
                    if (any_rej) {
                        for (int i = lane; i < N; i += 64) skey[i] &= KEYMASK;
                        wk = wk == 0xFFFFFFFFu ? wk : (wk & KEYMASK);
                        any_rej = 0;
                    }
                    c = rl32(vc, off);
                    ctopo = TOPO_ON && (d.cls_flags[c] & CF_TOPO) != 0;
                    tl = rl64(vtol, off);
#pragma unroll
                    for (int ai = 0; ai < KP_LDS_AXES; ai++) pq[ai] = rl32(vq[ai], off);
                    if (lane < R) S.shape_req[lane] = qw_req[off * R + lane];
                    wa = wb >= 0 && wb + lane < N && absorbed(wm);
                    sstart = 0;
                    prev_shape = shape;
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                }
                // ExistingNode.Add on the existing nodes in order, before sort.Slice (no re-sort when one accepts); a
                // pod of a topology class is placed on existing nodes by the block (domain counts, node requirements)
                if (d.E > 0 && xstart < d.E && !(TOPO_ON && ctopo)) {
                    int jf = -1;
                    for (int base = xstart; base < d.E; base += 64) {
                        const int j = base + lane;
                        bool cand = false;
                        if (j < d.E) {
                            const uint64_t xw = __hip_atomic_load(&d.XT[(size_t)c * d.EW + (j >> 6)], __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT);
                            cand = (xw >> (j & 63)) & 1ull;
#pragma unroll
                            for (int ai = 0; ai < KP_MAX_R; ai++) {
                                if (ai < d.n_active) {
                                    const int64_t pr = S.shape_req[d.active_axes[ai]];
                                    const int64_t h = ld_req(&d.ex_head[(size_t)ai * d.E + j]) - (j == xj ? pr * xcnt : 0);
                                    cand &= pr <= h;
                                }
                            }
                        }
                        const uint64_t m = ballot(cand);
                        if (m) {
                            jf = base + __ffsll((unsigned long long)m) - 1;
                            break;
                        }
                    }
                    if (jf >= 0) {
                        if (jf != xj) ex_flush();
                        xj = jf;
                        xcnt++;
                        if (d.ex_mayfix) {
                            ex_flush();
                            existing_merge(d, jf, c, lane);
                        }
                        if (lane == 0) {
                            d.pod_result[p] = -2 - jf;
                            d.pod_order[p] = seq;
                        }
                        seq++;
                        xstart = jf;
                        nexist++;
                        continue;
                    }
                    ex_flush();
                    xstart = d.E;
                }
                if (TOPO_ON && ctopo && (dkind || eager) && d.E > 0) {
                    // the slice sort (or the block's eager move becoming Go's) waits for the block's existing-node
                    // pass (topo_defer above)
                    win_flush();
                    wb = -1;
                    if (lane < R) S.pod_req[lane] = qw_req[off * R + lane];
                    if (lane == 0) {
                        S.cur_pod = p;
                        S.cls_fill = S.CC.cls != c;
                        S.topo_pod = 1;
                        S.topo_defer = 1;
                        S.topo_exdone = 0;
                    }
                    break;
                }
              }
                scanned += N;
                const long long t_b = prof_clock(d);
                cqpop += t_b - t_a;
                // sort.Slice(s.newNodeClaims, by len(Pods)) at the start of add(): at most one element changed since
                // the last sort (dkind 1: position dpos gained a pod; dkind 2: a NodeClaim was appended)
                eager = 0;  // this add() sorts: the eager move is now Go's too
                if (dkind) {
                    int how = 0;
                    bool done_here = false;
                    if (dkind == 1 && wb >= 0 && dpos >= wb && dpos < wb + 64) {
                        // in the window: key[f] (already incremented) moves to the end of its old run
                        const int f = dpos;
                        uint32_t kv = (uint32_t)rl32((int)wk, f - wb) & KEYMASK;
                        uint64_t ge = ballot(wb + lane > f && (wb + lane >= N || (wk & KEYMASK) >= kv));
                        if (ge == 0 && wb + 64 < N && wb != f) {  // the run leaves the window: re-base it at f
                            win_flush();
                            win_load(f);
                            ge = ballot(wb + lane > f && (wb + lane >= N || (wk & KEYMASK) >= kv));
                        }
                        const int fl = f - wb, q = wb + lane;
                        const bool in_window = ge != 0 || wb + 64 >= N;
                        const int el = ge ? __ffsll((unsigned long long)ge) - 1 : N - wb;  // run end e - wb
                        if (el == fl + 1) {
                            n_noinv++;
                            done_here = true;  // key[f+1] >= key[f]: no inversion
                        } else if (in_window) {
                            bool fast = N <= 12;
                            if (!fast && N >= 50) {
                                fast = !is_pivot_sample(N, f);
                                if (!fast) {
                                    n_pivot++;
                                    win_flush();
                                    fast = choose_pivot_hint_wave(sl, N, lane) == 1;
                                }
                            }
                            if (fast) {
                                // stable move: [f, e-1) <- [f+1, e), e-1 <- the changed element (registers move along)
                                const bool sh = lane >= fl && lane < el - 1, last = lane == el - 1;
                                auto mv = [&](auto& x) {
                                    using X = std::remove_reference_t<decltype(x)>;
                                    const int xf = rl32((int)x, fl);
                                    // lane i ← lane i+1 with a DPP wavefront shift (wave_shl:1) instead of an LDS
                                    // permute; lane 63's result is unused (sh requires lane < el - 1 <= 63)
                                    const int nx = __builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xF, 0xF, false);
                                    x = sh ? (X)nx : (last ? (X)xf : x);
                                };
                                mv(wk);
                                mv(wo);
                                mv(wm);
                                mv(wcnt);
#pragma unroll
                                for (int ai = 0; ai < KP_LDS_AXES; ai++) mv(wh[ai]);
                                {
                                    int wai = wa ? 1 : 0;
                                    mv(wai);
                                    wa = wai != 0;
                                }
                                how = 1;
                                n_winmove++;
                                done_here = true;
                            }
                        }
                    }
                    if (!done_here) {
                        n_ldssort++;
                        if (dkind == 2) n_r2++;
                        else if (wb < 0) n_rwb++;
                        else if (!(dpos >= wb && dpos < wb + 64)) n_rout++;
                        win_flush();
                        how = sort_slice_after_change(sl, N, dkind, dpos, S.sstack, lane);
                        wb = -1;
                    }
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    sfast += how == 1;
                    sfull += how == 2;
                    const long long c1 = prof_clock(d);
                    csort += c1 - t_b;
                    if (how == 2) csfull += c1 - t_b;
                    // positions < dpos are untouched by a stable move of dpos and rejected this shape (when the
                    // shape repeats); an append or a full pdqsort permutes everything
                    if (dkind == 2 || how == 2 || sstart > dpos) sstart = 0;
                    dkind = 0;
                }
                if (TOPO_ON && ctopo) {
                    // a pod with topology terms: the block handles it (topology prefilter, quick accept with
                    // recording, or the evaluation of candidates); counts change with every placement
                    win_flush();
                    wb = -1;
                    if (off >= 0 && lane < R) S.pod_req[lane] = qw_req[off * R + lane];
                    if (lane == 0) {
                        S.cur_pod = p;
                        S.cls_fill = S.CC.cls != c;
                        S.topo_pod = 1;
                        S.topo_exdone = off < 0;  // a resumed pod: no existing node took it
                    }
                    break;
                }
                // first NodeClaim in slice order (from sstart) that has not rejected this shape
                const long long t_c = prof_clock(d);
                int f = N;
                for (int pos = sstart; pos < N;) {
                    if (wb < 0 || pos < wb || pos >= wb + 64) {
                        win_flush();
                        win_load(pos);
                    }
                    const int q = wb + lane;
                    const uint64_t m = ballot(q >= pos && !(wk >> 31));  // positions >= N carry bit 31
                    if (m) {
                        f = wb + __ffsll((unsigned long long)m) - 1;
                        break;
                    }
                    pos = wb + 64;
                }
                const long long t_d = prof_clock(d);
                cqscan += t_d - t_c;
                if (f < N) {
                    const int fl = f - wb;
                    bool wfit = A > 0;  // no witness table (A == 0): every pod is evaluated
#pragma unroll
                    for (int ai = 0; ai < KP_LDS_AXES; ai++)
                        if (ai < A) wfit &= pq[ai] <= wh[ai];
                    uint64_t okm = ballot(wa && wfit);
                    if ((KP_NOOP_RESV | !RESV) && !((okm >> fl) & 1ull) && ((ballot(wfit) >> fl) & 1ull) && d.noop_quick) {
                        // the NodeClaim at f has not absorbed the class but its witness fits: the Add is the quick accept
                        // when the class's requirement merge changes nothing (and the class tolerates its template)
                        const int nc = rl32((int)wo, fl), tm = (int)((uint32_t)rl32((int)wm, fl) >> 16);
                        if (((tl >> tm) & 1ull) && merge_noop(d, S, nc, c, lane)) {
                            if (lane == fl) {
                                wm = (wm & 0xFFFF0000u) | (uint32_t)(uint16_t)c;
                                wa = true;
                            }
                            if (lane == 0) {
                                slast[nc] = (uint16_t)c;  // its requirements are a subset of the class's
                                if (d.profile) S.st[ST_SLOW_WHY + 4]++;
                            }
                            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                            okm |= 1ull << fl;
                        }
                    }
                    if ((okm >> fl) & 1ull) {
                        // quick accept: NodeClaim.Add(pod) succeeds with state (requirements, options) unchanged.
                        // Batch: the next pods of the same shape go one each to the following NodeClaims of the run of
                        // equal len(Pods) starting at f (each placement moves the NodeClaim at f to the end of the run,
                        // so pod i meets the run's i-th element at f), as long as each of them quick-accepts, each move
                        // is pdqsort's stable move (no choosePivot sample at f), and the run ends inside the window.
                        const uint32_t kk = (uint32_t)rl32((int)wk, fl);  // len(Pods) at f, rejected bit clear
                        int m = 1;
                        const bool movable = N <= 12 || (N >= 50 && !is_pivot_sample(N, f));
                        uint64_t ge = ballot(wb + lane > f && (wb + lane >= N || (wk & KEYMASK) > kk));
                        uint64_t okm2 = okm;
                        int fl2 = fl;
                        if (movable && ge == 0 && fl > 0 && qw_used < qw_n && xstart >= d.E) {
                            // the run leaves the window: re-base the window at f to batch over up to 64 of its elements
                            win_flush();
                            win_load(f);
                            bool ok2 = wa && A > 0;
#pragma unroll
                            for (int ai = 0; ai < KP_LDS_AXES; ai++)
                                if (ai < A) ok2 &= pq[ai] <= wh[ai];
                            okm2 = ballot(ok2);
                            fl2 = 0;
                            ge = ballot(wb + lane > f && (wb + lane >= N || (wk & KEYMASK) > kk));
                        }
                        const int fl = fl2;
                        const uint64_t okm = okm2;
                        const int el = ge ? __ffsll((unsigned long long)ge) - 1 : 64;  // run end (lane), 64: beyond window
                        if (movable && qw_used < qw_n && (el < 64 || fl == 0) && xstart >= d.E) {
                            // same-shape pods queued right after this one (lastLen termination checked per pod)
                            const int q0 = qcount + 1;  // len(queue) when this pod was popped
                            const uint64_t sm = ballot(lane >= off && lane < qw_n && vshape == shape &&
                                                       vlast != q0 - (lane - off));
                            const int np = __builtin_ctzll(~(sm >> off));
                            // run elements from f on that are not rejected and quick-accept
                            const uint64_t tm = okm & ~ballot((wk >> 31) != 0) & (ge ? (ge - 1) : ~0ull);
                            const int nt = __builtin_ctzll(~(tm >> fl));
                            m = np < nt ? np : nt;
                            if (m > 64) m = 64;
                        }
                        // lanes fl .. fl+m-1 take pods off .. off+m-1
                        const int pi = lane - fl;
                        const bool tgt = pi >= 0 && pi < m;
                        const int podl = __shfl(vp, (off + (pi < 0 ? 0 : pi)) & 63);
                        if (tgt) {
#pragma unroll
                            for (int ai = 0; ai < KP_LDS_AXES; ai++) wh[ai] -= pq[ai];
                            wk += 1;
                            wcnt += 1;
                            d.pod_result[podl] = (int)wo;
                            d.pod_order[podl] = seq + pi;
                        }
                        if (m > 1 && el == 64) {
                            // the run [f, e) continues past the window: write the window back, then permute in LDS:
                            // [f, e) becomes elem_{m-1}, elem_m .. elem_{L-1}, elem_{m-2} .. elem_0
                            const uint32_t mk = wk, mo = wo;  // lanes < m: the placed elements (keys incremented)
                            win_flush();
                            int e = N;
                            for (int base = f + 64; base < N; base += 64) {
                                const int qq = base + lane;
                                const uint64_t gm = ballot(qq >= N || (skey[qq < N ? qq : 0] & KEYMASK) > kk);
                                if (gm) {
                                    e = base + __ffsll((unsigned long long)gm) - 1;
                                    break;
                                }
                            }
                            if (e > N) e = N;
                            // [f+m, e) -> [f+1, e-m+1), ascending chunks (each chunk is read before it is overwritten)
                            for (int base = f + m; base < e; base += 64) {
                                const int qq = base + lane;
                                uint32_t kx = 0;
                                uint16_t ox = 0;
                                if (qq < e) {
                                    kx = skey[qq];
                                    ox = sord[qq];
                                }
                                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                                if (qq < e) {
                                    skey[qq - (m - 1)] = kx;
                                    sord[qq - (m - 1)] = ox;
                                }
                                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                            }
                            if (lane == m - 1) {
                                skey[f] = mk;
                                sord[f] = (uint16_t)mo;
                            } else if (lane < m - 1) {
                                skey[e - 1 - lane] = mk;
                                sord[e - 1 - lane] = (uint16_t)mo;
                            }
                            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                            wb = -1;
                            sfast += m - 1;
                            n_winmove += m - 1;
                            qw_used += m - 1;
                            qhead += m - 1;
                            if (qhead >= P) qhead -= P;
                            qcount -= m - 1;
                            popped += m - 1;
                            scanned += (long long)N * (m - 1);
                        } else if (m > 1) {
                            // apply the m-1 completed stable moves: [f, e) becomes
                            // elem_{m-1}, elem_m .. elem_{L-1}, elem_{m-2} .. elem_0   (elem_{m-1}'s move is pending)
                            int src = lane;
                            if (lane >= fl && lane < el) {
                                if (lane == fl) src = fl + m - 1;
                                else if (lane <= el - m) src = lane + m - 1;
                                else src = fl + el - 1 - lane;
                            }
                            wk = (uint32_t)__shfl((int)wk, src);
                            wo = (uint32_t)__shfl((int)wo, src);
                            wm = (uint32_t)__shfl((int)wm, src);
                            wcnt = __shfl(wcnt, src);
#pragma unroll
                            for (int ai = 0; ai < KP_LDS_AXES; ai++) wh[ai] = __shfl(wh[ai], src);
                            wa = __shfl(wa ? 1 : 0, src) != 0;
                            sfast += m - 1;
                            n_winmove += m - 1;
                            qw_used += m - 1;
                            qhead += m - 1;
                            if (qhead >= P) qhead -= P;
                            qcount -= m - 1;
                            popped += m - 1;
                            scanned += (long long)N * (m - 1);
                        }
                        seq += m;
                        dkind = 1;
                        dpos = f;
                        sstart = f;
                        nquick += m;
                        n_batch++;
                        const long long t_e = prof_clock(d);
                        cqcheck += t_e - t_d;
                        continue;
                    }
                }
                // slow path: the whole block evaluates this pod
                if (d.profile) {  // KPSIM_PROFILE: why the quick accept does not apply
                    const bool fa = f < N && rl32(wa ? 1 : 0, (f - wb) & 63) != 0;
                    if (lane == 0) S.st[ST_SLOW_WHY + (f >= N ? 0 : A == 0 ? 3 : !fa ? 1 : 2)]++;
                }
                win_flush();
                wb = -1;
                if (lane < R) S.pod_req[lane] = qw_req[off * R + lane];
                if (lane == 0) {
                    S.cur_pod = p;
                    S.cls_fill = S.CC.cls != c;  // decided before the barrier: fill_class_cache rewrites CC.cls
                    S.topo_pod = 0;
                }
                collect_candidates(d, S, skey, sord, stmpl, ~0ull, N, f, 0, lane);
                break;
            }
            win_flush();
            ex_flush();
            if (lane == 0) {
                S.xstart = xstart;
                S.st[ST_EXIST_PLACED] += nexist;
                S.qhead = qhead;
                S.qcount = qcount;
                S.seq = seq;
                S.prev_shape = prev_shape;
                S.dirty_kind = dkind;
                S.dirty_pos = dpos;
                S.scan_start = sstart;
                S.eager = eager;
                S.any_rej = any_rej;
                S.topo_resume = 0;
                // reset here, behind the barrier that opens the slow path: the winner wave reads it at its commit,
                // which no barrier separates from the end of the iteration
                S.rej_volatile = 0;
                S.done = done;
                S.err = err;
                S.cur_cls = c;
                S.cur_tol = tl;
                S.st[ST_POPPED] = popped;
                S.st[ST_NC_SCANNED] += scanned;
                S.st[ST_QUICK] += nquick;
                S.st[ST_SLOW] += done ? 0 : 1;
                S.st[ST_SORT_FAST] += sfast;
                S.st[ST_SORT_FULL] += sfull;
                S.st[ST_CYC_SORT] += csort;
                S.st[ST_CYC_SORT_FULL] += csfull;
                S.st[ST_CYC_QPOP] += cqpop;
                S.st[ST_CYC_QSCAN] += cqscan;
                S.st[ST_CYC_QCHECK] += cqcheck;
                S.st[ST_CYC_QCOMMIT] += cqcommit;
                S.st[ST_N_NOINV] += n_noinv;
                S.st[ST_N_WINMOVE] += n_winmove;
                S.st[ST_N_LDSSORT] += n_ldssort;
                S.st[ST_N_PIVOT] += n_pivot;
                S.st[ST_N_WINLOAD] += n_winload;
                S.st[ST_N_FLUSH] += n_flush;
                S.st[ST_N_SHAPE] += n_shape;
                S.st[ST_N_SHAPE + 1] += n_r2;
                S.st[ST_N_SHAPE + 2] += n_rwb;
                S.st[ST_N_SHAPE + 3] += n_rout;
                S.st[ST_N_SHAPE + 4] += n_batch;

                S.st[ST_CYC_POP] += prof_clock(d) - c_in;
            }
            if (lane < KP_LDS_AXES) {
#pragma unroll
                for (int ai = 0; ai < KP_LDS_AXES; ai++)
                    if (lane == ai) S.cur_pq[ai] = pq[ai];
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // flushed request totals have reached L2
        }
        __syncthreads();
        if (S.done) break;
        const long long c_slow = prof_clock(d);
        if (d.profile && tid == 0) S.st[ST_SEG + 0] += c_slow - c_top;
        const int pod = S.cur_pod;
        if (TOPO_ON && S.topo_pod && d.E > 0 && !S.topo_exdone) {
            // ================= a pod with topology terms: existing nodes first (wave 0) =================
            // ExistingNode.Add in scheduling order: tolerations + Compatible (XT) and headroom, then the requirement
            // merge and Topology.AddRequirements on the node's own domains; the first node that accepts takes the pod
            // and Topology.Record counts it there.  Counts change with every placement, so nothing is memoised.
            if (S.cls_fill) fill_class_cache<TOPO>(d, S.cur_cls, S.CC, tid, nthr, TOPO ? S.born : 0ull);
            __syncthreads();
            if (wave == 0) {
                const int placed = existing_topo_scan(d.self, S, pod, lane);
                if (lane == 0) {
                    S.ex_placed = placed;
                    S.cls_fill = 0;
                }
            }
            __syncthreads();
            if (S.ex_placed >= 0 || S.topo_defer) {
                if (tid == 0) {
                    S.tp_n = 0;
                    S.topo_pod = 0;
                    S.topo_resume = S.ex_placed < 0;  // no existing node took it: wave 0 sorts, then the NodeClaims
                    S.topo_defer = 0;
                }
                __syncthreads();
                continue;
            }
        }
        if (TOPO_ON && S.topo_pod) {
            // ================= a pod with topology terms (wave 0) =================
            // prefilter of this pod's groups, first surviving NodeClaim in slice order; quick accept when it has
            // absorbed the class, every narrowed key is a single admitted domain and the witness fits; otherwise
            // the block evaluates candidates from there
            const long long t0 = prof_clock(d);
            const int c = S.cur_cls, N = S.N;
            const uint32_t cfl = d.cls_flags[c];
            const int scan_from = S.scan_start;
            const uint64_t ctol = d.tol[c];
#if KP_TOPO_BLOCK_SCAN
            if (tid == 0) {
                S.tp_n = 0;
                S.tp_all = 1;
            }
            if (cfl & CF_TOPO_CONS) topo_prefilter_setup(d, S, c, wave, lane);
            __syncthreads();  // every group's entry and TopoSnap row
            if (tid == 0 && (cfl & CF_TOPO_CONS)) S.tp_cls = c;  // read by the next setup, behind the next slow-path barrier
            const long long t1 = prof_clock(d);
            const int f = topo_scan_block(d, S, skey, sord, stmpl, ctol, N, scan_from, S.bred, wave, lane);
#else
            int f = N;
            long long t1 = 0;
            if (wave == 0) {
                if (lane == 0) {
                    S.tp_n = 0;
                    S.tp_all = 1;
                }
                if (cfl & CF_TOPO_CONS)
                    for (int w = 0; w < KP_NWAVES; w++) topo_prefilter_setup(d, S, c, w, lane);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                t1 = prof_clock(d);
                f = topo_scan(d, S, skey, sord, stmpl, ctol, N, scan_from, lane);
            }
#endif
            const long long t2 = prof_clock(d);
            if (wave == 0) {
                bool quick = false;
                if (d.profile && lane == 0) {  // KPSIM_PROFILE: why the topology quick accept does not apply
                    const int nc = f < N ? sord[f] : 0;
                    const int why = f >= N ? 0 : !(cfl & CF_TOPO_QREC) ? 1 : nc >= NQ ? 2
                                  : !(slast[nc] == (uint16_t)c || ((cfl & CF_NOKEYS) && ((d.tol[c] >> stmpl[nc]) & 1ull))) ? 3 : 4;
                    S.st[ST_TQ_WHY + why]++;
                }
                if (f < N && (cfl & CF_TOPO_QREC) && A > 0 && S.tp_all) {
                    const int nc = sord[f], tm = stmpl[nc];
                    const bool absd = slast[nc] == (uint16_t)c || ((cfl & CF_NOKEYS) && ((d.tol[c] >> tm) & 1ull));
                    bool ok = nc < NQ;
                    for (int ai = 0; ai < A && ok; ai++) ok = S.cur_pq[ai] <= shr[ai * NQ + nc];
                    if (d.profile && lane == 0 && nc < NQ && ok) S.st[ST_TQ_WHY + 5]++;  // witness fits
                    ok = ok && topo_pinned(d, S, nc, lane);
                    // a NodeClaim that has not absorbed the class: quick when the Add's merge changes nothing
                    const bool noop = ok && !absd && merge_noop(d, S, nc, c, lane);
                    if (d.profile && lane == 0 && noop) S.st[ST_TQ_WHY + 6]++;
                    quick = ok && (absd || noop);
                    if (noop && lane == 0) slast[nc] = (uint16_t)c;  // its requirements are a subset of the class's
                    if (quick) {
                        if (lane < A) shr[lane * NQ + nc] -= S.cur_pq[lane];
                        if (lane < R && S.pod_req[lane])
                            atomicAdd((unsigned long long*)&d.nc_req[(size_t)nc * R + lane], (unsigned long long)S.pod_req[lane]);
                        topo_record_quick(d, S, c, nc, tm, S.born, lane);
                        if (lane == 0) {
                            skey[f]++;
                            d.pod_result[pod] = nc;
                            d.pod_order[pod] = S.seq++;
                            S.dirty_kind = 1;
                            S.dirty_pos = f;
                            S.scan_start = 0;
                            S.st[ST_TOPO_QUICK]++;
                            S.st[ST_QUICK]++;
                        }
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                }
                if (!quick) collect_candidates(d, S, skey, sord, stmpl, ctol, N, f, 0, lane);
                if (lane == 0) {
                    S.topo_quick = quick;
                    if (quick) {  // nothing reads these before the next slow-path entry (behind wave 0's fast loop)
                        S.tp_n = 0;
                        S.topo_pod = 0;
                    }
                    if (d.profile) {
                        S.st[ST_CYC_TSETUP] += t1 - t0;
                        S.st[ST_CYC_TSCAN] += t2 - t1;
                    }
                }
            }
            __syncthreads();
            if (S.topo_quick) {
                if (d.profile && tid == 0) {
                    S.st[ST_TQ_ITERS]++;
                    S.st[ST_TQ_CYC] += __builtin_amdgcn_s_memtime() - c_slow;
                }
                continue;
            }
        }
        long long c_ev0 = 0;
        {
            const long long cf0 = (d.profile && tid == 0) ? __builtin_amdgcn_s_memtime() : 0;
            if (S.cls_fill) fill_class_cache<TOPO>(d, S.cur_cls, S.CC, tid, nthr, TOPO ? S.born : 0ull);
            if (d.profile && tid == 0) {
                c_ev0 = __builtin_amdgcn_s_memtime();
                S.st[ST_SLOW_WHY + 10] += c_ev0 - cf0;
                S.st[ST_SEG + 1] += cf0 - c_slow;
                S.st[ST_SEG + 2] += c_ev0 - cf0;
            }
        }

        // ================= in-flight NodeClaims in slice order: first whose Add succeeds =================
        int round = 0, win = -1;
        // a pod with topology terms: its candidates one at a time, each evaluated by the whole block (the type sweep
        // split over the waves; the first candidate that passes the prefilter usually accepts), in slice order
        const bool team = TOPO_ON && S.topo_pod && d.team_eval;
        if (d.trace && pod == d.trace_pod && wave == 0) {  // diagnostics: the slice as the slow path sees it
            int* sl = d.trace + 1 + 6 * KP_TRACE_N;
            if (lane == 0) {
                sl[0] = S.N;
                sl[1] = S.scan_start;
                sl[2] = S.cand_pos[0][0];
            }
            for (int i = lane; i < S.N && i < 4096; i += 64) {
                sl[3 + 2 * i] = sord[i];
                sl[4 + 2 * i] = (int)skey[i];
            }
        }
        for (int ti = 0; team;) {
            const int b = round & 1;
            const int n = S.n_cand[b];
            for (int i = 0; i < n; i++, ti++) {
                const int nc = sord[S.cand_pos[b][i]];
                EvalIn a;
                a.Ahdr = d.nc_hdr + (size_t)nc * K;
                a.Aw = d.nc_words + (size_t)nc * d.DW;
                a.opts = lane < TW ? d.nc_opts[(size_t)nc * TW + lane] : 0;
                a.base_req = d.nc_req + (size_t)nc * R;
                a.pod_req = S.pod_req;
                a.tmpl = d.nc_tmpl[nc];
                a.compat = true;
                a.force_off = false;
                a.prof = (d.profile && wave == 0) ? &S.st[ST_EV_REQ] : nullptr;
                a.host = d.E + nc;
                a.held = (RESV && d.resv_on) ? held_word(d, nc, lane) : 0ull;
                // the buffer by the joins reached so far, not by candidate index: a candidate rejected before the join
                // (no barrier) must not flip the parity
                TeamBuf* const tb = &S.team[tjoins & 1];
                const bool ok = (S.CC.flags & CF_TOPO_CONS)
                                    ? eval_wave<true, RESV, true, PREF, false, true>(d, E, S.CC, a, S.ws[wave], lane, tb,
                                                                                     wave, KP_NWAVES, &tjoins)
                                    : eval_wave<false, RESV, true, PREF, false, true>(d, E, S.CC, a, S.ws[wave], lane,
                                                                                      tb, wave, KP_NWAVES, &tjoins);
                if (wave == 0 && lane == 0) {
                    S.fastp[b][i] = 0;
                    S.acc[b][i] = ok;
                    if (!ok && S.ws[0].memo_ok) {  // as below: rejected this shape for good
                        skey[S.cand_pos[b][i]] |= 0x80000000u;
                        S.any_rej = 1;
                    }
                    if (!ok && !S.ws[0].memo_ok) S.rej_volatile = 1;
                    S.st[ST_NC_EVALS]++;
                }
                if (ok) {
                    win = i;
                    break;
                }
            }
            if (win >= 0 || S.scan_done[b]) break;
            if (wave == 0)
                collect_candidates(d, S, skey, sord, stmpl, S.topo_pod ? d.tol[S.cur_cls] : ~0ull, S.N, S.scan_next[b], b ^ 1, lane);
            __syncthreads();
            round++;
        }
        // a pod without topology terms whose first candidate needs the full Add (it has not absorbed the class): that
        // candidate first, evaluated by the whole block (it takes most such pods); the others then in parallel as below
        int first = 0;  // round-0 candidates already evaluated
        bool team_won = false;
        if ((KP_TEAM_FIRST_RESV | !RESV) && (KP_TEAM_FIRST_TOPO | !TOPO))
        if (!team && d.team_first && S.n_cand[0] > 0) {
            const int nc = sord[S.cand_pos[0][0]];
            const int tm = d.nc_tmpl[nc];
            const bool fast0 = !(S.CC.flags & CF_TOPO) && !(RESV && d.resv_on && ld_i32(&d.nc_rlive[nc])) &&
                               (slast[nc] == (uint16_t)S.cur_cls || ((S.CC.flags & CF_NOKEYS) && ((S.CC.tol >> tm) & 1ull)));
            if (!fast0) {
                EvalIn a;
                a.Ahdr = d.nc_hdr + (size_t)nc * K;
                a.Aw = d.nc_words + (size_t)nc * d.DW;
                a.opts = lane < TW ? d.nc_opts[(size_t)nc * TW + lane] : 0;
                a.base_req = d.nc_req + (size_t)nc * R;
                a.pod_req = S.pod_req;
                a.tmpl = tm;
                a.compat = true;
                a.force_off = false;
                a.prof = (d.profile && wave == 0) ? &S.st[ST_EV_REQ] : nullptr;
                a.host = d.E + nc;
                a.held = (RESV && d.resv_on) ? held_word(d, nc, lane) : 0ull;
                TeamBuf* const tb = &S.team[tjoins & 1];
                const bool ok = (TOPO_ON && (S.CC.flags & CF_TOPO_CONS))
                                    ? eval_wave<true, RESV, true, PREF, false, true>(d, E, S.CC, a, S.ws[wave], lane, tb,
                                                                                     wave, KP_NWAVES, &tjoins)
                                    : eval_wave<false, RESV, true, PREF, false, true>(d, E, S.CC, a, S.ws[wave], lane,
                                                                                      tb, wave, KP_NWAVES, &tjoins);
                if (wave == 0 && lane == 0) {
                    S.fastp[0][0] = 0;
                    S.acc[0][0] = ok;
                    if (!ok && S.ws[0].memo_ok) {
                        skey[S.cand_pos[0][0]] |= 0x80000000u;
                        S.any_rej = 1;
                    }
                    if (!ok && !S.ws[0].memo_ok) S.rej_volatile = 1;
                    S.st[ST_NC_EVALS]++;
                    if (d.profile) S.st[ST_SLOW_WHY + 8]++;
                }
                first = 1;
                if (ok) {
                    win = 0;
                    team_won = true;
                }
                __syncthreads();  // the team's scratch and acc[0][0] before the parallel round
            }
        }
        for (; !team && !team_won;) {
            const int b = round & 1;
            const int f0 = round == 0 ? first : 0;  // candidate index of wave 0
            const int ci = wave + f0;
            if (ci < S.n_cand[b]) {
                const int nc = sord[S.cand_pos[b][ci]];
                EvalIn a;
                a.Ahdr = d.nc_hdr + (size_t)nc * K;
                a.Aw = d.nc_words + (size_t)nc * d.DW;
                a.opts = lane < TW ? d.nc_opts[(size_t)nc * TW + lane] : 0;
                a.base_req = d.nc_req + (size_t)nc * R;
                a.pod_req = S.pod_req;
                a.tmpl = d.nc_tmpl[nc];
                a.compat = true;
                a.force_off = false;
                a.prof = d.profile ? &S.st[ST_EV_REQ] : nullptr;
                a.host = d.E + nc;
                a.held = (RESV && d.resv_on) ? held_word(d, nc, lane) : 0ull;
                // a NodeClaim that keeps reserved offerings re-runs the whole Add (its reservations are recomputed)
                const bool fast = !(S.CC.flags & CF_TOPO) && !(RESV && d.resv_on && ld_i32(&d.nc_rlive[nc])) &&
                                  (slast[nc] == (uint16_t)S.cur_cls || ((S.CC.flags & CF_NOKEYS) && ((S.CC.tol >> a.tmpl) & 1ull)));
                if (fast && lane == 0) S.ws[wave].memo_ok = 1;
                const bool ok = fast ? eval_fits_only<PREF>(d, E, a, S.ws[wave], lane)
                                : (TOPO_ON && (S.CC.flags & CF_TOPO_CONS)) ? eval_wave<true, RESV, true, PREF>(d, E, S.CC, a, S.ws[wave], lane)
                                                              : eval_wave<false, RESV, true, PREF>(d, E, S.CC, a, S.ws[wave], lane);
                if (d.trace && (pod == d.trace_pod || (S.cur_cls == -2 - d.trace_pod && pod <= d.trace_max)) && lane == 0) {
                    const int i = atomicAdd(&d.trace[0], 1);
                    {  // ring of the last KP_TRACE_N entries
                        int* e = d.trace + 1 + 6 * (i % KP_TRACE_N);
                        e[0] = pod;
                        e[1] = nc;
                        e[2] = ok;
                        e[3] = S.ws[wave].memo_ok | (fast << 1) | ((RESV ? ld_i32(&d.nc_rlive[nc]) : 0) << 2);
                        e[4] = S.cand_pos[b][ci];
                        e[5] = (int)(rl64(a.held, 0) & 0xFFFFFFFFu);
                    }
                }
                if (lane == 0) {
                    S.fastp[b][ci] = fast;
                    S.acc[b][ci] = ok;
                    if (!ok && S.ws[wave].memo_ok) {
                        // rejected this shape for good (positions are stable here); a rejection that depended on
                        // topology counts is not memoised, one that depended on reservation capacity until rel_flag
                        skey[S.cand_pos[b][ci]] |= 0x80000000u;
                        S.any_rej = 1;
                    }
                    if (!ok && !S.ws[wave].memo_ok) S.rej_volatile = 1;
                    if (fast) atomicAdd((unsigned long long*)&S.st[ST_WITNESS_MISS], 1ull);
                }
            }
            __syncthreads();
            const int nc_ = S.n_cand[b];
            for (int w = f0; w < nc_; w++)
                if (S.acc[b][w]) {
                    win = w;
                    break;
                }
            if (tid == 0) S.st[ST_NC_EVALS] += nc_ > f0 ? nc_ - f0 : 0;
            if (win >= 0 || S.scan_done[b]) break;
            if (wave == 0)
                collect_candidates(d, S, skey, sord, stmpl, S.topo_pod ? d.tol[S.cur_cls] : ~0ull, S.N, S.scan_next[b], b ^ 1, lane);
            __syncthreads();
            round++;
        }
        long long c_ev = 0;
        if (tid == 0 && d.profile) {
            const long long t1 = __builtin_amdgcn_s_memtime();
            S.st[ST_CYC_SCAN] += t1 - c_slow;
            S.st[ST_SEG + 3] += t1 - c_ev0;
            c_ev = t1;
        }
        if (d.profile && tid == 0 && !S.topo_pod)  // KPSIM_PROFILE: where the slow path's pods land
            S.st[ST_SLOW_WHY + (win < 0 ? 7 : (round == 0 && win == 0) ? 5 : 6)]++;
        if (win >= 0) {
            // the wave whose scratch holds the accepted Add (team: every wave's does)
            const int cw = (team || team_won) ? 0 : win - (round == 0 ? first : 0);
            if (wave == cw) {
                const int pos = S.cand_pos[round & 1][win];
                const int nc = sord[pos];
                if (!S.fastp[round & 1][win]) {
                    commit_reqs(d, S.CC, S.ws[cw], nc, lane);
                    if (RESV && d.resv_on) commit_reservations(d, sRcap, S.ws[cw], nc, false, &S.rel_flag, lane);
                }
                if (PREF && d.best_effort) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // commit_reqs' header rows have landed
                    commit_min_relax(d, S.ws[cw], nc, lane);
                }
                if (TOPO_ON && (S.CC.flags & CF_TOPO))
                    topo_record(d, S.CC, S.ws[cw], d.nc_hdr + (size_t)nc * K, d.nc_words + (size_t)nc * d.DW,
                                d.E + nc, d.nc_tmpl[nc], true, lane, -1, nullptr, S.born);
                if (lane < TW) d.nc_opts[(size_t)nc * TW + lane] = S.ws[cw].opts[lane];
                if (lane < R && S.pod_req[lane])
                    atomicAdd((unsigned long long*)&d.nc_req[(size_t)nc * R + lane], (unsigned long long)S.pod_req[lane]);
                if (lane < A && nc < NQ) shr[lane * NQ + nc] = S.ws[cw].hr[lane];
                if (lane == 0) {
                    slast[nc] = (uint16_t)S.cur_cls;
                    skey[pos]++;
                    S.dirty_kind = 1;
                    S.dirty_pos = pos;
                    // every position before the winner rejected this shape for good, unless rejections depended on
                    // topology counts (not memoised; the next pod of the shape rescans them)
                    S.scan_start = ((S.CC.flags & CF_TOPO) || S.rej_volatile) ? 0 : pos;
                    if (d.trace && S.cur_cls == -2 - d.trace_pod && pod <= d.trace_max) {
                        const int i = atomicAdd(&d.trace[0], 1);
                        {
                            int* e = d.trace + 1 + 6 * (i % KP_TRACE_N);
                            e[0] = pod;
                            e[1] = -1000 - nc;
                            e[2] = S.scan_start;
                            e[3] = S.rej_volatile;
                            e[4] = pos;
                            e[5] = 0;
                        }
                    }
                    d.pod_result[pod] = nc;
                    d.pod_order[pod] = S.seq++;
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        } else {
            // ================= new NodeClaim from the templates (NodePool weight order) =================
            const long long c_t = prof_clock(d);
            // NewNodeClaim(template jj) for the pod, by wave cw (whose scratch holds the template's accepted Add)
            auto commit_tmpl = [&](int jj, int cw) {
                const int n = S.N;
                // NewNodeClaim(template): requirements = template requirements, then the Add's merge
                for (int k = lane; k < K; k += 64) d.nc_hdr[(size_t)n * K + k] = d.cls_hdr[(size_t)(d.C + jj) * K + k];
                for (int i = lane; i < d.DW; i += 64)
                    d.nc_words[(size_t)n * d.DW + i] = d.cls_words[(size_t)(d.C + jj) * d.DW + i];
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                commit_reqs(d, S.CC, S.ws[cw], n, lane);
                if (PREF && d.best_effort) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the header rows above have landed
                    commit_min_relax(d, S.ws[cw], n, lane);
                }
                if (RESV && d.resv_on) commit_reservations(d, sRcap, S.ws[cw], n, true, &S.rel_flag, lane);
                if (TOPO_ON && (S.CC.flags & CF_TOPO))
                    topo_record(d, S.CC, S.ws[cw], d.cls_hdr + (size_t)(d.C + jj) * K,
                                d.cls_words + (size_t)(d.C + jj) * d.DW, d.E + n, jj, true, lane, -1, nullptr,
                                S.born);
                if (lane < TW) d.nc_opts[(size_t)n * TW + lane] = S.ws[cw].opts[lane];
                for (int r = lane; r < R; r += 64)
                    __hip_atomic_store(&d.nc_req[(size_t)n * R + r], d.daemon[(size_t)jj * R + r] + S.pod_req[r],
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (lane < A && n < NQ) shr[lane * NQ + n] = S.ws[cw].hr[lane];
                // subtractMax(remaining, nodeClaim.InstanceTypeOptions)
                for (int r = 0; r < R; r++) {
                    if (!d.limit_set[(size_t)jj * R + r]) continue;
                    int64_t mx = INT64_MIN;
                    for (int w2 = 0; w2 < TW; w2++) {
                        const uint64_t ow = S.ws[cw].opts[w2];
                        if ((ow >> lane) & 1ull) {
                            const int64_t cp = d.cap[(size_t)r * T + w2 * 64 + lane];
                            mx = cp > mx ? cp : mx;
                        }
                    }
                    mx = wave_max64(mx);
                    if (lane == 0) d.remaining[(size_t)jj * R + r] -= mx;
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the new remaining limits have landed
                limit_mask_update(d, jj, lane);
                if (lane == 0) {
                    slast[n] = (uint16_t)S.cur_cls;
                    stmpl[n] = (uint8_t)jj;
                    d.nc_tmpl[n] = jj;
                    sord[n] = (uint16_t)n;
                    skey[n] = 1;
                    S.N = n + 1;
                    S.dirty_kind = 2;
                    S.dirty_pos = n;
                    d.pod_result[pod] = n;
                    d.pod_order[pod] = S.seq++;
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            };
            int twin = -1;
            if (KP_TEAM_TMPL && (!RESV || KP_TEAM_TMPL_RESV) && !TOPO && d.team_first) {
                // the templates one at a time in weight order, each evaluated by the whole block (the type sweep split
                // over the waves, as for a team candidate): the first that accepts wins, and every wave's scratch holds
                // its Add
                for (int j = 0; j < d.NT; j++) {
                    uint64_t o = (lane < TW && d.tmpl_ok[j]) ? d.tmpl_opts[(size_t)j * TW + lane] : 0;
                    o = limit_filter(d, j, o, lane);
                    if (!ballot(o != 0)) continue;  // the same for every wave
                    EvalIn a;
                    a.Ahdr = d.cls_hdr + (size_t)(d.C + j) * K;
                    a.Aw = d.cls_words + (size_t)(d.C + j) * d.DW;
                    a.opts = o;
                    a.base_req = d.daemon + (size_t)j * R;
                    a.pod_req = S.pod_req;
                    a.tmpl = j;
                    a.compat = true;
                    a.force_off = false;
                    a.prof = nullptr;
                    a.host = d.E + S.N;  // NewNodeClaim's fresh hostname (no pod counted there yet)
                    a.held = 0;
                    TeamBuf* const tbuf = &S.team[tjoins & 1];
                    const bool ok = (TOPO_ON && (S.CC.flags & CF_TOPO_CONS))
                                        ? eval_wave<true, RESV, true, PREF, false, true>(d, E, S.CC, a, S.ws[wave], lane, tbuf,
                                                                                         wave, KP_NWAVES, &tjoins)
                                        : eval_wave<false, RESV, true, PREF, false, true>(d, E, S.CC, a, S.ws[wave], lane,
                                                                                          tbuf, wave, KP_NWAVES, &tjoins);
                    if (tid == 0) S.st[ST_TMPL_EVALS]++;
                    if (ok) {
                        twin = j;
                        break;
                    }
                }
                if (twin >= 0 && (S.N >= NCMAX || S.N >= d.NCcap)) {
                    if (tid == 0) S.err = 1;
                    twin = -1;
                }
                if (twin >= 0 && wave == 0) commit_tmpl(twin, 0);
            } else
            for (int tb = 0; tb < d.NT; tb += KP_NWAVES) {
                const int j = tb + wave;
                if (j < d.NT) {
                    uint64_t o = (lane < TW && d.tmpl_ok[j]) ? d.tmpl_opts[(size_t)j * TW + lane] : 0;
                    o = limit_filter(d, j, o, lane);
                    bool ok = false;
                    if (ballot(o != 0)) {
                        EvalIn a;
                        a.Ahdr = d.cls_hdr + (size_t)(d.C + j) * K;
                        a.Aw = d.cls_words + (size_t)(d.C + j) * d.DW;
                        a.opts = o;
                        a.base_req = d.daemon + (size_t)j * R;
                        a.pod_req = S.pod_req;
                        a.tmpl = j;
                        a.compat = true;
                        a.force_off = false;
                        a.prof = nullptr;
                        a.host = d.E + S.N;  // NewNodeClaim's fresh hostname (no pod counted there yet)
                        a.held = 0;
                        ok = (TOPO_ON && (S.CC.flags & CF_TOPO_CONS)) ? eval_wave<true, RESV, true, PREF>(d, E, S.CC, a, S.ws[wave], lane)
                                                         : eval_wave<false, RESV, true, PREF>(d, E, S.CC, a, S.ws[wave], lane);
                    }
                    if (d.trace && pod == d.trace_pod && lane == 0) {
                        const int i = atomicAdd(&d.trace[0], 1);
                        {
                            int* e = d.trace + 1 + 6 * (i % KP_TRACE_N);
                            e[0] = -1;
                            e[1] = -1 - j;
                            e[2] = ok;
                            e[3] = S.ws[wave].memo_ok;
                            e[4] = e[5] = 0;
                        }
                    }
                    if (lane == 0) S.tacc[wave] = ok;
                }
                __syncthreads();
                for (int w = 0; w < KP_NWAVES && tb + w < d.NT; w++)
                    if (S.tacc[w]) {
                        twin = w;
                        break;
                    }
                if (tid == 0) S.st[ST_TMPL_EVALS] += (d.NT - tb < KP_NWAVES ? d.NT - tb : KP_NWAVES);
                if (twin >= 0 && (S.N >= NCMAX || S.N >= d.NCcap)) {
                    if (tid == 0) S.err = 1;
                    twin = -1;
                    break;
                }
                if (twin >= 0) {
                    if (wave == twin) {
                        const int jj = tb + wave;
                        const int n = S.N;
                        // NewNodeClaim(template): requirements = template requirements, then the Add's merge
                        for (int k = lane; k < K; k += 64) d.nc_hdr[(size_t)n * K + k] = d.cls_hdr[(size_t)(d.C + jj) * K + k];
                        for (int i = lane; i < d.DW; i += 64)
                            d.nc_words[(size_t)n * d.DW + i] = d.cls_words[(size_t)(d.C + jj) * d.DW + i];
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        commit_reqs(d, S.CC, S.ws[wave], n, lane);
                        if (PREF && d.best_effort) {
                            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the header rows above have landed
                            commit_min_relax(d, S.ws[wave], n, lane);
                        }
                        if (RESV && d.resv_on) commit_reservations(d, sRcap, S.ws[wave], n, true, &S.rel_flag, lane);
                        if (TOPO_ON && (S.CC.flags & CF_TOPO))
                            topo_record(d, S.CC, S.ws[wave], d.cls_hdr + (size_t)(d.C + jj) * K,
                                        d.cls_words + (size_t)(d.C + jj) * d.DW, d.E + n, jj, true, lane, -1, nullptr,
                                        S.born);
                        if (lane < TW) d.nc_opts[(size_t)n * TW + lane] = S.ws[wave].opts[lane];
                        for (int r = lane; r < R; r += 64)
                            __hip_atomic_store(&d.nc_req[(size_t)n * R + r], d.daemon[(size_t)jj * R + r] + S.pod_req[r],
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (lane < A && n < NQ) shr[lane * NQ + n] = S.ws[wave].hr[lane];
                        // subtractMax(remaining, nodeClaim.InstanceTypeOptions)
                        for (int r = 0; r < R; r++) {
                            if (!d.limit_set[(size_t)jj * R + r]) continue;
                            int64_t mx = INT64_MIN;
                            for (int w2 = 0; w2 < TW; w2++) {
                                const uint64_t ow = S.ws[wave].opts[w2];
                                if ((ow >> lane) & 1ull) {
                                    const int64_t cp = d.cap[(size_t)r * T + w2 * 64 + lane];
                                    mx = cp > mx ? cp : mx;
                                }
                            }
                            mx = wave_max64(mx);
                            if (lane == 0) d.remaining[(size_t)jj * R + r] -= mx;
                        }
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the new remaining limits have landed
                        limit_mask_update(d, jj, lane);
                        if (lane == 0) {
                            slast[n] = (uint16_t)S.cur_cls;
                            stmpl[n] = (uint8_t)jj;
                            d.nc_tmpl[n] = jj;
                            sord[n] = (uint16_t)n;
                            skey[n] = 1;
                            S.N = n + 1;
                            S.dirty_kind = 2;
                            S.dirty_pos = n;
                            d.pod_result[pod] = n;
                            d.pod_order[pod] = S.seq++;
                        }
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                    break;
                }
                __syncthreads();  // tacc is rewritten by the next template batch
            }
            if (tid == 0) {
                if (d.profile) S.st[ST_CYC_TMPL] += __builtin_amdgcn_s_memtime() - c_t;
                if (twin < 0) {  // preferences.Relax, then Queue.Push(pod, relaxed)
                    const int tail = (S.qhead + S.qcount) % P;
                    d.qbuf[tail] = pod;
                    S.qcount++;
                    const int nx = (PREF && d.relax_next) ? d.relax_next[S.cur_cls] : -1;
                    if (nx >= 0) {
                        // the pod takes its class's next relaxation stage (Topology.Update / updateCachedPodData) and
                        // lastLen is cleared: a new epoch
                        d.pod_cls[pod] = nx;
                        d.pod_shape[pod] = d.shape_next[S.prev_shape];
                        S.epoch++;
                        S.relaxed = 1;
                        if (d.tg_late) S.born = topo_birth(d, S.born, d.cls_birth[nx]);  // Topology.Update: the spec's new groups
                    } else {
                        d.last_len[pod] = S.qcount;
                        if (PREF && d.last_ep) d.last_ep[pod] = S.epoch;
                    }
                }
            }
        }
        if (d.block_sort) {
            __syncthreads();  // the commit's slice change (key, dirty_kind / dirty_pos) is visible
            block_sort_move(S, sl, tid, nthr);
        }
        if (tid == 0) {
            S.tp_n = 0;
            S.topo_pod = 0;
        }
        __syncthreads();
        if (tid == 0 && d.profile) {  // commit / templates
            S.st[ST_SLOW_WHY + 9] += __builtin_amdgcn_s_memtime() - c_ev;
            S.st[ST_SEG + 4] += __builtin_amdgcn_s_memtime() - c_ev;
        }
    }

    if (S.eager && wave == 0) {  // no add() sorted after the last eager move: undo it (rotate [pos, e) right by one)
        const int a = S.eager_pos, e = S.eager_e;
        const uint32_t lk = skey[e - 1];
        const uint16_t lo = sord[e - 1];
        for (int top = e - 1; top > a; top -= 64) {  // descending chunks: each is read before it is overwritten
            const int i = top - lane;
            uint32_t k = 0;
            uint16_t o = 0;
            if (i > a) {
                k = skey[i - 1];
                o = sord[i - 1];
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            if (i > a) {
                skey[i] = k;
                sord[i] = o;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        if (lane == 0) {
            skey[a] = lk;
            sord[a] = lo;
        }
    }
    __syncthreads();

    // ---- outputs ----
    const int N = S.N;
    for (int i = tid; i < N; i += nthr) {
        d.nc_npods[sord[i]] = (int32_t)(skey[i] & KEYMASK);
        d.nc_slice_pos[sord[i]] = i;
    }
    if (tid == 0) {
        d.nc_count[0] = N;
        d.err[0] = S.err;
        for (int i = 0; i < ST_COUNT; i++) d.stats[i] = S.st[i];
    }
}

}  // namespace KP_WNS
using namespace KP_WNS;
