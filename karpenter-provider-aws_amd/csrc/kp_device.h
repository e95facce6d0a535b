// kp_device.h — device helpers: requirement-digest algebra on u64 value bitsets.
//
// Restates, over dictionary bitsets, the [core] scheduling.Requirement operations the scheduler uses
// (sigs.k8s.io/karpenter pkg/scheduling/requirement.go: Intersection, Len, Operator, Has, withinIntPtrs;
// requirements.go: Compatible, Intersects).  A digest key is {ReqHdr, nw[k] words}; bit v of the words is
// value id v of key k.  Sets are exact because every value a solve can mention is in the dictionary.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kp_layout.h"

#define OP_IN 0
#define OP_NOTIN 1
#define OP_EXISTS 2
#define OP_DNE 3

__device__ __forceinline__ uint64_t rl64(uint64_t x, int lane) {
    uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, lane);
    uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(x >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int rl32(int x, int lane) { return __builtin_amdgcn_readlane(x, lane); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// KpDev's small arrays are read with constant indices only: a runtime index into the by-value kernel argument makes
// the compiler copy the whole struct to scratch.  These select the element through a compare chain instead.
__device__ __forceinline__ int act_axis(const KpDev& d, int ai) {
    int r = 0;
#pragma unroll
    for (int i = 0; i < KP_MAX_R; i++)
        if (i == ai) r = d.active_axes[i];
    return r;
}
__device__ __forceinline__ int qshift_of(const KpDev& d, int ai) {
    int r = 0;
#pragma unroll
    for (int i = 0; i < KP_LDS_AXES; i++)
        if (i == ai) r = d.qshift[i];
    return r;
}

// Requirement.Operator() of a DEFINED requirement with `nvals` values
__device__ __forceinline__ int req_op(uint32_t flags, int nvals) {
    if (flags & RF_CMP) return nvals > 0 ? OP_NOTIN : OP_EXISTS;
    return nvals > 0 ? OP_IN : OP_DNE;
}
__device__ __forceinline__ bool op_notin_or_dne(int op) { return op == OP_NOTIN || op == OP_DNE; }

// A type's reserved-offering rows as bits of their ResvTab word (KpDev::type_ro packing: word << 16 | first << 8 | n).
__device__ __forceinline__ uint64_t ro_span_bits(uint32_t tr) {
    const uint32_t n = tr & 255u, b = (tr >> 8) & 255u;
    return n == 0 ? 0ull : ((n >= 64 ? ~0ull : ((1ull << n) - 1ull)) << b);
}
// 64-bit __shfl (per-lane source lane)
__device__ __forceinline__ uint64_t shfl64(uint64_t x, int src) {
    return ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(x >> 32), src) << 32) | (uint32_t)__shfl((int)(uint32_t)x, src);
}

// withinIntPtrs(value, gt, lt)
__device__ __forceinline__ bool within(const KpDev& d, int k, int v, const ReqHdr& h) {
    if (!(h.flags & (RF_GT | RF_LT))) return true;
    int b = d.vbase[k] + v;
    if (!d.val_isint[b]) return false;
    int64_t x = d.val_int[b];
    if ((h.flags & RF_GT) && h.gt >= x) return false;
    if ((h.flags & RF_LT) && h.lt <= x) return false;
    return true;
}

// Requirement.Has(value) for a DEFINED requirement
__device__ __forceinline__ bool req_has(const KpDev& d, int k, int v, const ReqHdr& h, const uint64_t* w) {
    bool bit = (w[v >> 6] >> (v & 63)) & 1ull;
    if (h.flags & RF_CMP) return !bit && within(d, k, v, h);
    return bit && within(d, k, v, h);
}

__device__ __forceinline__ int popc_words(const uint64_t* w, int n) {
    int c = 0;
    for (int i = 0; i < n; i++) c += __popcll(w[i]);
    return c;
}

// Is Requirement.Intersection(A, B) empty (Len() == 0)?  Count-free form of req_intersect, single lane.
__device__ inline bool req_intersect_empty(const KpDev& d, int k, const ReqHdr& A, const uint64_t* aw, const ReqHdr& B,
                                           const uint64_t* bw) {
    const bool ac = A.flags & RF_CMP, bc = B.flags & RF_CMP;
    const bool hg = (A.flags | B.flags) & RF_GT, hl = (A.flags | B.flags) & RF_LT;
    ReqHdr o;
    o.flags = (hg ? RF_GT : 0u) | (hl ? RF_LT : 0u);
    o.gt = 0;
    o.lt = 0;
    o.minv = 0;
    if (hg) o.gt = ((A.flags & RF_GT) && (B.flags & RF_GT)) ? (A.gt > B.gt ? A.gt : B.gt) : ((A.flags & RF_GT) ? A.gt : B.gt);
    if (hl) o.lt = ((A.flags & RF_LT) && (B.flags & RF_LT)) ? (A.lt < B.lt ? A.lt : B.lt) : ((A.flags & RF_LT) ? A.lt : B.lt);
    if (hg && hl && o.gt >= o.lt) return true;  // DoesNotExist
    if (ac && bc) return false;                 // complement: Len = MaxInt64 - |values|
    const int n = d.nw[k];
    for (int i = 0; i < n; i++) {
        uint64_t x;
        if (ac) x = bw[i] & ~aw[i];
        else if (bc) x = aw[i] & ~bw[i];
        else x = aw[i] & bw[i];
        if (hg || hl) {
            uint64_t y = x;
            while (y) {
                const int jb = __ffsll((unsigned long long)y) - 1;
                y &= y - 1;
                if (!within(d, k, i * 64 + jb, o)) x &= ~(1ull << jb);
            }
        }
        if (x) return false;
    }
    return true;
}

// Requirements.Compatible(node, podRequirements) with no undefined-label allowance (ExistingNode.Add), single lane:
// every key of pod class c must be defined on the node unless its operator is NotIn/DoesNotExist, and the
// intersection must be non-empty unless both operators are NotIn/DoesNotExist.
__device__ inline bool node_compatible(const KpDev& d, const ReqHdr* nh, const uint64_t* nwords, int c) {
    for (int i = d.cls_xkoff[c]; i < d.cls_xkoff[c + 1]; i++) {
        const int k = d.cls_xkeys[i];
        const ReqHdr B = d.cls_hdr[(size_t)c * d.K + k];
        const uint64_t* bw = d.cls_words + (size_t)c * d.DW + d.woff[k];
        const bool bno = op_notin_or_dne(req_op(B.flags, popc_words(bw, d.nw[k])));
        const ReqHdr A = nh[k];
        if (!(A.flags & RF_DEF)) {
            if (!bno) return false;
            continue;
        }
        const uint64_t* aw = nwords + d.woff[k];
        if (req_intersect_empty(d, k, A, aw, B, bw) && !(bno && op_notin_or_dne(req_op(A.flags, popc_words(aw, d.nw[k])))))
            return false;
    }
    return true;
}

// O = A ∩ B (Requirement.Intersection), single lane.  Returns |O.values|.
__device__ inline int req_intersect(const KpDev& d, int k, const ReqHdr& A, const uint64_t* aw, const ReqHdr& B,
                                    const uint64_t* bw, ReqHdr& O, uint64_t* ow) {
    const int n = d.nw[k];
    const bool ac = A.flags & RF_CMP, bc = B.flags & RF_CMP;
    const bool cmp = ac && bc;
    ReqHdr o;
    o.flags = RF_DEF | (cmp ? RF_CMP : 0u);
    o.gt = 0;
    o.lt = 0;
    bool hg = (A.flags | B.flags) & RF_GT, hl = (A.flags | B.flags) & RF_LT;
    if (hg) {
        if ((A.flags & RF_GT) && (B.flags & RF_GT)) o.gt = A.gt > B.gt ? A.gt : B.gt;
        else o.gt = (A.flags & RF_GT) ? A.gt : B.gt;
        o.flags |= RF_GT;
    }
    if (hl) {
        if ((A.flags & RF_LT) && (B.flags & RF_LT)) o.lt = A.lt < B.lt ? A.lt : B.lt;
        else o.lt = (A.flags & RF_LT) ? A.lt : B.lt;
        o.flags |= RF_LT;
    }
    o.minv = 0;
    if ((A.flags | B.flags) & RF_MIN) {
        o.flags |= RF_MIN;
        if ((A.flags & RF_MIN) && (B.flags & RF_MIN)) o.minv = A.minv > B.minv ? A.minv : B.minv;
        else o.minv = (A.flags & RF_MIN) ? A.minv : B.minv;
    }
    if (hg && hl && o.gt >= o.lt) {  // → DoesNotExist
        O.flags = RF_DEF | (o.flags & RF_MIN);
        O.minv = o.minv;
        O.gt = O.lt = 0;
        for (int i = 0; i < n; i++) ow[i] = 0;
        return 0;
    }
    int cnt = 0;
    for (int i = 0; i < n; i++) {
        uint64_t a = aw[i], b = bw[i], x;
        if (ac && bc) x = a | b;
        else if (ac) x = b & ~a;
        else if (bc) x = a & ~b;
        else x = a & b;
        if (hg || hl) {
            uint64_t y = x;
            while (y) {
                int j = __ffsll((unsigned long long)y) - 1;
                y &= y - 1;
                if (!within(d, k, i * 64 + j, o)) x &= ~(1ull << j);
            }
        }
        ow[i] = x;
        cnt += __popcll(x);
    }
    if (!cmp) {  // remove boundaries for concrete sets
        o.flags &= ~(RF_GT | RF_LT);
        o.gt = o.lt = 0;
    }
    O = o;
    return cnt;
}

// Node requirement A = B ∩ A in place (Requirements.Add of one pod requirement), single lane.  Returns whether A changed.
__device__ inline bool req_merge_inplace(const KpDev& d, int k, ReqHdr& A, uint64_t* aw, const ReqHdr& B,
                                         const uint64_t* bw) {
    const int n = d.nw[k];
    if (!(A.flags & RF_DEF)) {
        A = B;
        for (int i = 0; i < n; i++) aw[i] = bw[i];
        return true;
    }
    ReqHdr O;
    uint64_t tmp[KP_MAX_SCR_WORDS];
    const int nn = n < KP_MAX_SCR_WORDS ? n : KP_MAX_SCR_WORDS;
    req_intersect(d, k, B, bw, A, aw, O, tmp);
    bool ch = O.flags != A.flags || O.minv != A.minv || O.gt != A.gt || O.lt != A.lt;
    for (int i = 0; i < nn; i++) {
        ch |= tmp[i] != aw[i];
        aw[i] = tmp[i];
    }
    A = O;
    return ch;
}
