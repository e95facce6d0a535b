// kp_kernels.hip — gfx950 kernels of the scheduling simulation (no MFMA: bitset / gather / compare work).
//
//   class_mask_kernel     pod-class × instance-type label compatibility sweep (V bitsets): one wave per
//                         (class, 64-type word), ballot over lanes.  Reference: compatible(it, reqs) =
//                         it.Requirements.Intersects(reqs) ([core] scheduling/nodeclaim.go
//                         filterInstanceTypesByRequirements; called at pkg/providers/instance/filter/filter.go:53).
//   template_init_kernel  NewScheduler's NodeClaimTemplate.InstanceTypeOptions =
//                         filterInstanceTypesByRequirements(instanceTypes[np], nct.Requirements, {}, {}, {}).
//   ffd_kernel            Scheduler.Solve: the whole first-fit-decreasing loop in ONE workgroup (8 waves), the
//                         queue, Go sort.Slice emulation, NodeClaim.Add for up to 8 candidate NodeClaims at once,
//                         new-NodeClaim creation from templates with NodePool limits.
//   finalize_kernel       FinalizeScheduling + InstanceTypes.Truncate(reqs, 60) (OrderByPrice, minValues),
//                         one workgroup per NodeClaim.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kp_device.h"
#include "kp_eval.h"
#include "kp_gosort.h"
#include "kp_layout.h"

// ------------------------------------------------------------------------------------------------
// class × type label compatibility
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void class_mask_kernel(KpDev d) {
    const int w = blockIdx.x, c = blockIdx.y, lane = threadIdx.x;
    const int t = w * 64 + lane;
    bool bit = t < d.T;
    const int k0 = d.cls_koff[c], k1 = d.cls_koff[c + 1];
    for (int i = k0; i < k1 && bit; i++) {
        const int k = d.cls_keys[i];
        if (!(d.kflags[k] & KF_CAT_SINGLE)) continue;
        const uint16_t v = d.type_val[(size_t)d.kcat[k] * d.T + t];
        if (v >= VAL_ABSENT) continue;  // DoesNotExist types are handled by dne_mask at evaluation
        const ReqHdr h = d.cls_hdr[(size_t)c * d.K + k];
        bit = req_has(d, k, v, h, d.cls_words + (size_t)c * d.DW + d.woff[k]);
    }
    const uint64_t m = ballot(bit);
    if (lane == 0) d.V[(size_t)c * d.TW + w] = m;
}

// ------------------------------------------------------------------------------------------------
// NodeClaimTemplate.InstanceTypeOptions (NewScheduler): one wave per template
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void template_init_kernel(KpDev d) {
    __shared__ ClassCache CC;
    __shared__ WaveScratch ws;
    __shared__ Roles roles;
    const int j = blockIdx.x, lane = threadIdx.x;
    fill_class_cache(d, d.C + j, CC, lane, 64);
    if (lane < 5) {
        const int rk = lane == 0 ? d.key_zone : lane == 1 ? d.key_ct : lane == 2 ? d.key_zoneid : lane == 3 ? d.key_resvid : d.key_resvtype;
        roles.key[lane] = rk;
        roles.woff[lane] = rk >= 0 ? d.woff[rk] : 0;
        roles.nw[lane] = rk >= 0 ? d.nw[rk] : 0;
    }
    __syncthreads();
    EvalEnv E;
    E.alloc = nullptr;  // no requests: Fits({}, alloc) only needs non-negative allocatable (tmpl rows ∧ nonneg)
    E.astride = 0;
    E.avail = d.avail_zc;
    E.multi16 = nullptr;
    E.slot_zone = d.slot_zone;
    E.slot_ct = d.slot_ct;
    E.slot_zoneid = d.slot_zoneid;
    E.roles = &roles;
    E.min_tmpl_mask = d.min_keys[(size_t)j * KP_MAX_CLASS_KEYS] >= 0 ? (1u << j) : 0u;
    EvalIn a;
    a.Ahdr = d.empty_hdr;
    a.Aw = d.empty_words;
    a.opts = lane < d.TW ? (d.tmpl_rows[(size_t)j * d.TW + lane] & d.nonneg[lane]) : 0;
    a.base_req = nullptr;
    a.pod_req = nullptr;
    a.tmpl = j;
    a.compat = false;
    a.force_off = true;
    a.prof = nullptr;
    const bool ok = eval_wave(d, E, CC, a, ws, lane);
    if (lane < d.TW) d.tmpl_opts[(size_t)j * d.TW + lane] = ok ? ws.opts[lane] : 0;
    if (lane == 0) d.tmpl_ok[j] = ok ? 1 : 0;
}

// ------------------------------------------------------------------------------------------------
// Solve: single-workgroup first-fit-decreasing
// ------------------------------------------------------------------------------------------------
// Fixed part of the FFD kernel's LDS.  The variable-size tables follow it at the offsets of the LDS plan
// (kp_ffd_plan_lds): slice keys/order and last absorbed class per NodeClaim, the staged allocatable / offering /
// multi-valued label tables, and the quick-accept headroom table hr[lds_A][lds_nq].
struct FfdShared {
    uint32_t rej[KP_MAX_NC / 32];  // NodeClaims that rejected the current pod shape (valid until they change)
    int qw_pod[64], qw_cls[64], qw_shape[64], qw_last[64];  // queue prefetch window
    int64_t qw_req[64][KP_MAX_R];
    int fastp[2][KP_NWAVES];
    WaveScratch ws[KP_NWAVES];
    ClassCache CC;
    Roles roles;
    int slot_zone[KP_MAX_SLOTS], slot_ct[KP_MAX_SLOTS], slot_zoneid[KP_MAX_SLOTS];
    int64_t pod_req[KP_MAX_R];
    int cand_pos[2][KP_NWAVES];
    int acc[2][KP_NWAVES];
    int tacc[KP_NWAVES];
    int n_cand[2], scan_done[2], scan_next[2];
    int sstack[64 * 5];
    // control state: owned by wave 0 inside its fast loop, by the block between the slow-path barriers
    int N, qhead, qcount, qw_base, qw_n, qw_used, done, cur_pod, cur_cls, cur_shape, prev_shape;
    int dirty_kind, dirty_pos, seq, err, cls_fill;
    long long st[ST_COUNT];
};

// wave 0: collect up to KP_NWAVES slice positions >= start whose NodeClaim has not rejected the current shape
__device__ inline void collect_candidates(FfdShared& S, const uint16_t* ord, int N, int start, int buf, int lane) {
    int cnt = 0, pos = start, next = N;
    while (pos < N) {
        const int p = pos + lane;
        bool c = false;
        if (p < N) {
            const int nc = ord[p];
            c = !((S.rej[nc >> 5] >> (nc & 31)) & 1u);
        }
        const uint64_t m = __ballot(c);
        const int rank = cnt + __popcll(m & ((1ull << lane) - 1ull));
        if (c && rank < KP_NWAVES) S.cand_pos[buf][rank] = p;
        const int tot = cnt + __popcll(m);
        if (tot >= KP_NWAVES) {
            const uint64_t last = __ballot(c && rank == KP_NWAVES - 1);
            next = pos + __ffsll((unsigned long long)last);  // position after the last collected candidate
            cnt = KP_NWAVES;
            break;
        }
        cnt = tot;
        pos += 64;
    }
    if (lane == 0) {
        S.n_cand[buf] = cnt;
        S.scan_next[buf] = cnt == KP_NWAVES ? next : N;
        S.scan_done[buf] = (cnt < KP_NWAVES) || next >= N;
    }
}

// types whose Capacity exceeds a NodePool's remaining limits (filterByRemainingResources)
__device__ inline uint64_t limit_filter(const KpDev& d, int j, uint64_t o, int lane) {
    bool any_limit = false;
    for (int r = 0; r < d.R; r++) any_limit |= d.limit_set[(size_t)j * d.R + r] != 0;
    if (!any_limit) return o;
    uint64_t out = 0;
    for (int w = 0; w < d.TW; w++) {
        const uint64_t cw = rl64(o, w);
        if (!cw) continue;
        const int t = w * 64 + lane;
        bool keep = (cw >> lane) & 1ull;
        if (keep) {
            for (int r = 0; r < d.R; r++)
                if (d.limit_set[(size_t)j * d.R + r] && d.cap[(size_t)r * d.T + t] > d.remaining[(size_t)j * d.R + r])
                    keep = false;
        }
        const uint64_t nb = ballot(keep);
        if (lane == w) out = nb;
    }
    return out;
}

__device__ __forceinline__ long long prof_clock(const KpDev& d) { return d.profile ? __builtin_amdgcn_s_memtime() : 0; }

// Scheduler.Solve.  Wave 0 runs the queue, the sort.Slice emulation and the first-fit scan for as many pods as it
// can resolve alone: a pod whose first non-rejected NodeClaim (slice order) has already absorbed the pod's class
// and whose witness type still fits is placed without an evaluation (exact: see pick_witness).  Any other pod is
// handed to all 8 waves (the slow path: NodeClaim.Add of up to 8 candidates at once, or the templates).
__global__ __launch_bounds__(KP_NWAVES * 64) void ffd_kernel(KpDev d) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    FfdShared& S = *reinterpret_cast<FfdShared*>(smem);
    uint32_t* const skey = reinterpret_cast<uint32_t*>(smem + d.off_key);   // len(Pods) by slice position
    uint16_t* const sord = reinterpret_cast<uint16_t*>(smem + d.off_ord);   // NodeClaim id by slice position
    uint16_t* const slast = reinterpret_cast<uint16_t*>(smem + d.off_last); // last absorbed class by NodeClaim id
    int64_t* const sAlloc = reinterpret_cast<int64_t*>(smem + d.off_alloc);
    uint64_t* const sAvail = reinterpret_cast<uint64_t*>(smem + d.off_avail);
    uint16_t* const sMulti = reinterpret_cast<uint16_t*>(smem + d.off_multi);
    int32_t* const shr = reinterpret_cast<int32_t*>(smem + d.off_hr);       // [A][NQ] witness headroom
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nthr = blockDim.x;
    const int T = d.T, TW = d.TW, K = d.K, R = d.R, P = d.P;
    const int TP = d.lds_tpad, NQ = d.lds_nq, A = d.lds_A, NCMAX = d.lds_ncmax;
    // ---- stage the type tables in LDS ----
    for (int i = tid; i < d.lds_nstage * TP; i += nthr) {
        const int ai = i / TP, t = i % TP;
        sAlloc[i] = t < T ? d.alloc[(size_t)d.active_axes[ai] * T + t] : 0;
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
    for (int i = tid; i < KP_MAX_NC / 32; i += nthr) S.rej[i] = 0;
    for (int p = tid; p < P; p += nthr) {
        d.qbuf[p] = d.queue0[p];
        d.last_len[p] = 0;
        d.pod_result[p] = -1;
        d.pod_order[p] = -1;
    }
    if (tid == 0) {
        S.N = 0;
        S.qhead = 0;
        S.qcount = P;
        S.qw_base = 0;
        S.qw_n = 0;
        S.qw_used = 0;
        S.done = 0;
        S.prev_shape = -1;
        S.dirty_kind = 0;
        S.dirty_pos = 0;
        S.seq = 0;
        S.err = 0;
        S.CC.cls = -1;
        S.cur_cls = -1;
        for (int i = 0; i < ST_COUNT; i++) S.st[i] = 0;
    }
    __syncthreads();
    EvalEnv E;
    E.alloc = sAlloc;
    E.astride = TP;
    E.avail = sAvail;
    E.multi16 = d.multi16 ? sMulti : nullptr;
    E.slot_zone = S.slot_zone;
    E.slot_ct = S.slot_ct;
    E.slot_zoneid = S.slot_zoneid;
    E.roles = &S.roles;
    {
        uint32_t mmask = 0;
        for (int j = 0; j < d.NT; j++)
            if (d.min_keys[(size_t)j * KP_MAX_CLASS_KEYS] >= 0) mmask |= 1u << j;
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

    for (;;) {
        // ================= wave 0: the fast loop =================
        if (wave == 0) {
            const long long c_in = prof_clock(d);
            const int N = S.N;
            int qhead = S.qhead, qcount = S.qcount, qw_n = S.qw_n, qw_used = S.qw_used;
            int seq = S.seq, prev_shape = S.prev_shape, dkind = S.dirty_kind, dpos = S.dirty_pos;
            int done = 0, err = S.err;
            long long popped = S.st[ST_POPPED], scanned = 0, nquick = 0, sfast = 0, sfull = 0, csort = 0;
            for (;;) {
                if (qcount == 0 || err) {
                    done = 1;
                    break;
                }
                if (popped > pop_bound) {  // a runaway loop is reported, not hung
                    err = 2;
                    done = 1;
                    break;
                }
                // Queue.Pop through an LDS window over the next <= 64 queue slots (pushes never land inside it)
                if (qw_used >= qw_n) {
                    const int wn = qcount < 64 ? qcount : 64;
                    if (lane < wn) {
                        int pos = qhead + lane;
                        if (pos >= P) pos -= P;
                        const int p = d.qbuf[pos];
                        S.qw_pod[lane] = p;
                        S.qw_cls[lane] = d.pod_cls[p];
                        S.qw_shape[lane] = d.pod_shape[p];
                        S.qw_last[lane] = d.last_len[p];
                        for (int r = 0; r < R; r++) S.qw_req[lane][r] = d.pod_req[(size_t)p * R + r];
                    }
                    qw_n = wn;
                    qw_used = 0;
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                }
                const int off = qw_used;
                if (S.qw_last[off] == qcount) {
                    done = 1;
                    break;
                }
                const int p = S.qw_pod[off], c = S.qw_cls[off], shape = S.qw_shape[off];
                qw_used++;
                qhead = qhead + 1 == P ? 0 : qhead + 1;
                qcount--;
                popped++;
                if (shape != prev_shape)
                    for (int i = lane; i < (NCMAX + 31) / 32; i += 64) S.rej[i] = 0;
                // sort.Slice(s.newNodeClaims, by len(Pods))
                const long long c0 = prof_clock(d);
                const int how = sort_slice_after_change(sl, N, dkind, dpos, S.sstack, lane);
                sfast += how == 1;
                sfull += how == 2;
                csort += prof_clock(d) - c0;
                dkind = 0;
                prev_shape = shape;
                scanned += N;
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                // first NodeClaim in slice order that has not rejected this shape
                int f = N;
                for (int base = 0; base < N; base += 64) {
                    const int q = base + lane;
                    bool cand = false;
                    if (q < N) {
                        const int nc = sord[q];
                        cand = !((S.rej[nc >> 5] >> (nc & 31)) & 1u);
                    }
                    const uint64_t m = ballot(cand);
                    if (m) {
                        f = base + __ffsll((unsigned long long)m) - 1;
                        break;
                    }
                }
                if (f < N) {
                    const int nc = sord[f];
                    if (nc < NQ && slast[nc] == (uint16_t)c) {
                        bool ok = true;
                        int64_t pq = 0;
                        if (lane < A) {
                            const int64_t pr = S.qw_req[off][my_axis];
                            pq = (pr + ((1ll << my_shift) - 1)) >> my_shift;
                            ok = pq <= (int64_t)shr[lane * NQ + nc];
                        }
                        if (ballot(!ok) == 0) {
                            // quick accept: NodeClaim.Add(pod) succeeds with state (requirements, options) unchanged
                            if (lane < A) shr[lane * NQ + nc] -= (int32_t)pq;
                            if (lane < R) {
                                const int64_t pr = S.qw_req[off][lane];
                                if (pr) atomicAdd((unsigned long long*)&d.nc_req[(size_t)nc * R + lane], (unsigned long long)pr);
                            }
                            if (lane == 0) {
                                skey[f]++;
                                d.pod_result[p] = nc;
                                d.pod_order[p] = seq;
                            }
                            seq++;
                            dkind = 1;
                            dpos = f;
                            nquick++;
                            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                            continue;
                        }
                    }
                }
                // slow path: the whole block evaluates this pod
                if (lane < R) S.pod_req[lane] = S.qw_req[off][lane];
                if (lane == 0) {
                    S.cur_pod = p;
                    S.cur_cls = c;
                    S.cur_shape = shape;
                    S.cls_fill = S.CC.cls != c;  // decided before the barrier: fill_class_cache rewrites CC.cls
                }
                collect_candidates(S, sord, N, f, 0, lane);
                break;
            }
            if (lane == 0) {
                S.qhead = qhead;
                S.qcount = qcount;
                S.qw_n = qw_n;
                S.qw_used = qw_used;
                S.seq = seq;
                S.prev_shape = prev_shape;
                S.dirty_kind = dkind;
                S.dirty_pos = dpos;
                S.done = done;
                S.err = err;
                S.st[ST_POPPED] = popped;
                S.st[ST_NC_SCANNED] += scanned;
                S.st[ST_QUICK] += nquick;
                S.st[ST_SLOW] += done ? 0 : 1;
                S.st[ST_SORT_FAST] += sfast;
                S.st[ST_SORT_FULL] += sfull;
                S.st[ST_CYC_SORT] += csort;
                S.st[ST_CYC_POP] += prof_clock(d) - c_in;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // quick-path atomics have reached L2
        }
        __syncthreads();
        if (S.done) break;
        const long long c_slow = prof_clock(d);
        const int pod = S.cur_pod;
        if (S.cls_fill) fill_class_cache(d, S.cur_cls, S.CC, tid, nthr);

        // ================= in-flight NodeClaims in slice order: first whose Add succeeds =================
        int round = 0, win = -1;
        for (;;) {
            const int b = round & 1;
            if (wave < S.n_cand[b]) {
                const int nc = sord[S.cand_pos[b][wave]];
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
                const bool fast = slast[nc] == (uint16_t)S.cur_cls;
                const bool ok = fast ? eval_fits_only(d, E, a, S.ws[wave], lane) : eval_wave(d, E, S.CC, a, S.ws[wave], lane);
                if (lane == 0) {
                    S.fastp[b][wave] = fast;
                    S.acc[b][wave] = ok;
                    if (!ok) atomicOr(&S.rej[nc >> 5], 1u << (nc & 31));
                    if (fast) S.st[ST_WITNESS_MISS]++;
                }
            }
            __syncthreads();
            const int nc_ = S.n_cand[b];
            for (int w = 0; w < nc_; w++)
                if (S.acc[b][w]) {
                    win = w;
                    break;
                }
            if (tid == 0) S.st[ST_NC_EVALS] += nc_;
            if (win >= 0 || S.scan_done[b]) break;
            if (wave == 0) collect_candidates(S, sord, S.N, S.scan_next[b], b ^ 1, lane);
            __syncthreads();
            round++;
        }
        if (tid == 0 && d.profile) {
            const long long t1 = __builtin_amdgcn_s_memtime();
            S.st[ST_CYC_SCAN] += t1 - c_slow;
        }
        if (win >= 0) {
            if (wave == win) {
                const int pos = S.cand_pos[round & 1][win];
                const int nc = sord[pos];
                if (!S.fastp[round & 1][win]) commit_reqs(d, S.CC, S.ws[win], nc, lane);
                if (lane < TW) d.nc_opts[(size_t)nc * TW + lane] = S.ws[win].opts[lane];
                if (lane < R && S.pod_req[lane])
                    atomicAdd((unsigned long long*)&d.nc_req[(size_t)nc * R + lane], (unsigned long long)S.pod_req[lane]);
                if (lane < A && nc < NQ) shr[lane * NQ + nc] = S.ws[win].hr[lane];
                if (lane == 0) {
                    slast[nc] = (uint16_t)S.cur_cls;
                    skey[pos]++;
                    S.dirty_kind = 1;
                    S.dirty_pos = pos;
                    d.pod_result[pod] = nc;
                    d.pod_order[pod] = S.seq++;
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        } else {
            // ================= new NodeClaim from the templates (NodePool weight order) =================
            const long long c_t = prof_clock(d);
            int twin = -1;
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
                        ok = eval_wave(d, E, S.CC, a, S.ws[wave], lane);
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
                        if (lane == 0) {
                            slast[n] = (uint16_t)S.cur_cls;
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
                if (twin < 0) {  // Queue.Push(pod, relaxed=false)
                    const int tail = (S.qhead + S.qcount) % P;
                    d.qbuf[tail] = pod;
                    S.qcount++;
                    d.last_len[pod] = S.qcount;
                }
            }
        }
        __syncthreads();
    }

    // ---- outputs ----
    const int N = S.N;
    for (int i = tid; i < N; i += nthr) {
        d.nc_npods[sord[i]] = (int32_t)skey[i];
        d.nc_slice_pos[sord[i]] = i;
    }
    if (tid == 0) {
        d.nc_count[0] = N;
        d.err[0] = S.err;
        for (int i = 0; i < ST_COUNT; i++) d.stats[i] = S.st[i];
    }
}

// ------------------------------------------------------------------------------------------------
// FinalizeScheduling + Truncate(OrderByPrice, maxInstanceTypes) + SatisfiesMinValues
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void finalize_kernel(KpDev d) {
    __shared__ uint64_t s_key[KP_MAX_TYPES];
    __shared__ uint32_t s_rank[KP_MAX_TYPES];
    __shared__ uint16_t s_t[KP_MAX_TYPES];
    __shared__ uint64_t s_mzc;
    __shared__ int s_n;
    __shared__ uint64_t s_bits[KP_MAX_MIN_WORDS];
    __shared__ int s_ok;
    __shared__ int64_t s_tot[KP_MAX_R];
    const int nc = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (nc >= d.nc_count[0]) return;
    const int T = d.T, TW = d.TW, M = d.M;
    const ReqHdr* H = d.nc_hdr + (size_t)nc * d.K;
    const uint64_t* W = d.nc_words + (size_t)nc * d.DW;
    if (tid == 0) {
        s_n = 0;
        s_ok = 1;
    }
    if (wave == 0) {
        // Offerings.Available().Compatible(reqs) over slots, reqs = NodeClaim requirements (hostname removed)
        bool ok = false;
        if (lane < d.n_slots) {
            auto adm = [&](int k, int v) -> bool {
                if (k < 0) return true;
                const ReqHdr h = H[k];
                if (!(h.flags & RF_DEF)) return true;
                return req_has(d, k, v, h, W + d.woff[k]);
            };
            auto dneok = [&](int k) -> bool {
                if (k < 0) return true;
                const ReqHdr h = H[k];
                if (!(h.flags & RF_DEF)) return true;
                return op_notin_or_dne(req_op(h.flags, popc_words(W + d.woff[k], d.nw[k])));
            };
            ok = adm(d.key_zone, d.slot_zone[lane]) && adm(d.key_ct, d.slot_ct[lane]) &&
                 (d.slot_zoneid[lane] < 0 || adm(d.key_zoneid, d.slot_zoneid[lane])) && dneok(d.key_resvid) &&
                 dneok(d.key_resvtype);
        }
        const uint64_t m = ballot(ok);
        if (lane == 0) s_mzc = m;
    }
    if (tid < d.R) s_tot[tid] = d.nc_req[(size_t)nc * d.R + tid];
    __syncthreads();
    const uint64_t mzc = s_mzc;
    for (int t = tid; t < TW * 64; t += blockDim.x) {
        if (t >= T) continue;
        if (!((d.nc_opts[(size_t)nc * TW + (t >> 6)] >> (t & 63)) & 1ull)) continue;
        // Fits(final requests, Allocatable): the quick-accept path applies Fits lazily (pick_witness)
        bool fit = true;
        for (int ai = 0; ai < d.n_active; ai++) {
            const int r = d.active_axes[ai];
            const int64_t tr = s_tot[r];
            if (tr > 0 && tr > d.alloc[(size_t)r * T + t]) fit = false;
        }
        if (!fit) continue;
        uint64_t m = d.avail_zc[t] & mzc;
        double price = 1.7976931348623157e308;  // math.MaxFloat64
        while (m) {
            const int s = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            const double p = d.slot_price[(size_t)t * KP_MAX_SLOTS + s];
            price = p < price ? p : price;
        }
        const int i = atomicAdd(&s_n, 1);
        s_key[i] = (uint64_t)__double_as_longlong(price);
        s_rank[i] = d.name_rank[t];
        s_t[i] = (uint16_t)t;
    }
    __syncthreads();
    const int n = s_n;
    for (int i = tid; i < n; i += blockDim.x) {
        const uint64_t ki = s_key[i];
        const uint32_t ri = s_rank[i];
        const uint16_t ti = s_t[i];
        int r = 0;
        for (int j = 0; j < n; j++) {
            const uint64_t kj = s_key[j];
            r += (kj < ki) || (kj == ki && (s_rank[j] < ri || (s_rank[j] == ri && s_t[j] < ti)));
        }
        if (r < M) d.nc_types[(size_t)nc * M + r] = ti;
    }
    if (tid == 0) {
        d.nc_nopts[nc] = n;
        d.nc_ntypes[nc] = n < M ? n : M;
    }
    __syncthreads();
    // Truncate: SatisfiesMinValues on the truncated list
    const int nt = n < M ? n : M;
    const int* mk = d.min_keys + (size_t)d.nc_tmpl[nc] * KP_MAX_CLASS_KEYS;
    for (int q = 0; q < KP_MAX_CLASS_KEYS; q++) {
        const int k = mk[q];
        if (k < 0) break;
        const ReqHdr h = H[k];
        if (!(h.flags & RF_MIN)) continue;
        for (int i = tid; i < KP_MAX_MIN_WORDS; i += blockDim.x) s_bits[i] = 0;
        __syncthreads();
        const int kc = d.kcat[k];
        for (int i = tid; i < nt; i += blockDim.x) {
            const int t = d.nc_types[(size_t)nc * M + i];
            if (kc < 0) continue;
            if (d.kflags[k] & KF_CAT_MULTI) {
                atomicOr((unsigned long long*)&s_bits[0], (unsigned long long)d.multi_mask[(size_t)d.kmulti[k] * T + t]);
            } else {
                const uint16_t v = d.type_val[(size_t)kc * T + t];
                if (v < VAL_ABSENT && v < KP_MAX_MIN_WORDS * 64)
                    atomicOr((unsigned long long*)&s_bits[v >> 6], 1ull << (v & 63));
            }
        }
        __syncthreads();
        if (tid == 0) {
            int c = 0;
            for (int i = 0; i < KP_MAX_MIN_WORDS; i++) c += __popcll(s_bits[i]);
            if (c < h.minv) s_ok = 0;
        }
        __syncthreads();
    }
    if (tid == 0) d.nc_valid[nc] = s_ok;
}

// ------------------------------------------------------------------------------------------------
// queue sort helpers (NewQueue: byCPUAndMemoryDescending, then creation time, then UID)
// ------------------------------------------------------------------------------------------------
__global__ void gather_key_kernel(const int64_t* __restrict__ field, int stride, int off, bool flip_desc,
                                  const int32_t* __restrict__ perm, uint64_t* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int p = perm[i];
    const int64_t v = field[(size_t)p * stride + off];
    uint64_t u = (uint64_t)v ^ 0x8000000000000000ull;  // order-preserving int64 → uint64
    if (flip_desc) u = ~u;
    out[i] = u;
}
__global__ void iota_kernel(int32_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = i;
}

// ------------------------------------------------------------------------------------------------
// launchers (called from kp_host.cpp)
// ------------------------------------------------------------------------------------------------
#include <hipcub/hipcub.hpp>

size_t kp_ffd_shared_bytes() { return sizeof(FfdShared); }

// Lay out the FFD kernel's dynamic LDS for this solve (fills d.off_*, d.lds_*).  Returns false if even the
// quick-accept-free layout exceeds max_bytes.
bool kp_ffd_plan_lds(KpDev& d, int max_bytes) {
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    size_t off = al(sizeof(FfdShared));
    const int ncmax = d.NCcap < KP_MAX_NC ? d.NCcap : KP_MAX_NC;
    d.lds_ncmax = ncmax;
    d.off_key = (int)off;
    off = al(off + 4 * (size_t)ncmax);
    d.off_ord = (int)off;
    off = al(off + 2 * (size_t)ncmax);
    d.off_last = (int)off;
    off = al(off + 2 * (size_t)ncmax);
    const int tp = (d.T + 63) / 64 * 64;
    d.lds_tpad = tp;
    d.lds_nstage = d.n_active < KP_LDS_AXES ? d.n_active : KP_LDS_AXES;
    d.off_alloc = (int)off;
    off = al(off + 8 * (size_t)d.lds_nstage * tp);
    d.off_avail = (int)off;
    off = al(off + 8 * (size_t)tp);
    d.off_multi = (int)off;
    if (d.multi16) off = al(off + 2 * (size_t)d.n_multi * tp);
    d.off_hr = (int)off;
    if ((int)off > max_bytes) return false;
    d.lds_A = d.n_active <= KP_LDS_AXES ? d.n_active : 0;
    int nq = 0;
    if (d.lds_A > 0) {
        nq = (int)((max_bytes - (int)off) / (4 * d.lds_A));
        nq = nq < ncmax ? nq : ncmax;
    }
    d.lds_nq = nq;
    if (nq == 0) d.lds_A = 0;
    off += 4 * (size_t)d.lds_A * nq;
    d.lds_bytes = (int)off;
    return true;
}

hipError_t kp_launch_class_mask(const KpDev& d, hipStream_t s) {
    dim3 g(d.TW, d.C + d.NT);
    hipLaunchKernelGGL(class_mask_kernel, g, dim3(64), 0, s, d);
    return hipGetLastError();
}
hipError_t kp_launch_template_init(const KpDev& d, hipStream_t s) {
    if (d.NT == 0) return hipSuccess;
    hipLaunchKernelGGL(template_init_kernel, dim3(d.NT), dim3(64), 0, s, d);
    return hipGetLastError();
}
hipError_t kp_launch_ffd(const KpDev& d, hipStream_t s) {
    static bool attr = false;
    const size_t bytes = (size_t)d.lds_bytes;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)ffd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, KP_LDS_BYTES);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL(ffd_kernel, dim3(1), dim3(KP_NWAVES * 64), bytes, s, d);
    return hipGetLastError();
}
hipError_t kp_launch_finalize(const KpDev& d, int n_nodeclaims, hipStream_t s) {
    if (n_nodeclaims <= 0) return hipSuccess;
    hipLaunchKernelGGL(finalize_kernel, dim3(n_nodeclaims), dim3(256), 0, s, d);
    return hipGetLastError();
}

// Stable LSD radix passes: uid key asc, creation asc, memory desc, cpu desc  →  queue0 (pod indices).
// fields: [P][4] int64 {cpu, mem, creation, uidkey^sign}.  tmp buffers owned by the caller.
hipError_t kp_queue_sort(const int64_t* fields, int n, int32_t* perm_a, int32_t* perm_b, uint64_t* keys_a,
                         uint64_t* keys_b, void* temp, size_t* temp_bytes, hipStream_t s, int32_t** result) {
    if (temp == nullptr) {
        size_t b = 0;
        hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, b, keys_a, keys_b, perm_a, perm_b, n, 0, 64, s);
        *temp_bytes = b;
        return e;
    }
    const int bs = 256, gs = (n + bs - 1) / bs;
    hipLaunchKernelGGL(iota_kernel, dim3(gs), dim3(bs), 0, s, perm_a, n);
    const int order[4] = {3, 2, 1, 0};
    const bool desc[4] = {false, false, true, true};
    int32_t* pin = perm_a;
    int32_t* pout = perm_b;
    for (int pass = 0; pass < 4; pass++) {
        hipLaunchKernelGGL(gather_key_kernel, dim3(gs), dim3(bs), 0, s, fields, 4, order[pass], desc[pass], pin, keys_a, n);
        size_t b = *temp_bytes;
        hipError_t e = hipcub::DeviceRadixSort::SortPairs(temp, b, keys_a, keys_b, pin, pout, n, 0, 64, s);
        if (e != hipSuccess) return e;
        int32_t* x = pin;
        pin = pout;
        pout = x;
    }
    *result = pin;
    return hipGetLastError();
}
