// kp_cons.h — device tables of a consolidation pass (kp_consolidate), shared by kp_host.cpp and kp_consolidate.hip.
//
// A probe is one SimulateScheduling + computeConsolidation ([core] pkg/controllers/disruption/helpers.go,
// consolidation.go): the probe's pods (pending + its candidates' reschedulable pods) are rescheduled onto every
// state node except its candidates, then onto at most one new NodeClaim (a second one makes the decision NONE, so
// the probe stops there).  One wave runs one probe; a persistent grid of waves pulls probes from a counter.
#pragma once
#include <stdint.h>

#include "../../include/kpsim.h"
#include "kp_layout.h"

enum { CS_POPS = 0, CS_EX_NODES, CS_NC_EVALS, CS_TMPL_EVALS, CS_PROBES, CS_BITMAP_WORDS, CS_PLACED_EXISTING,
       CS_NEW_NC, CS_CHUNK_LOADS, CS_CACHE_HITS, CS_CYC_BUILD, CS_CYC_SCAN, CS_CYC_NODECLAIM, CS_CYC_DECIDE,
       CS_CYC_TOTAL, CS_CHUNK_SKIPS, CS_RELAXED, CS_MUT, CS_COUNT = 18 };

#define KP_CONS_XTC 1024  // pod classes whose XT column of the cached node chunk is kept in LDS
#define KP_CONS_STORE 8   // node chunks the fast probe variant keeps in its LDS headroom store
#define KP_CONS_PP 16     // KPSIM_PROFILE: per-probe counters (kp_consolidate's diagnostics)
#define KP_CONS_FULL_WORKERS 1024  // FULL-variant workers: one per SIMD of 256 CUs (1 wave per SIMD at its VGPR count)

struct KpCons {
    int32_t n_probes;           // probes of this call (out[0 .. n_probes))
    int32_t probe0;             // first probe of the call (multi-node part for KP_CONSOLIDATE_BOTH)
    int32_t mode;               // KP_CONSOLIDATE_*
    int32_t n_multi;            // BOTH: out[0, n_multi) are multi-node probes probe0.., the rest single-node sprobe0..
    int32_t sprobe0;
    int32_t n_cand;
    int32_t spot_to_spot;
    int32_t v_spot, v_od;       // capacity-type value ids in the solve dictionary, -1 when absent
    uint64_t spot_slots;        // offering slots whose capacity type is spot / on-demand
    uint64_t od_slots;
    const int32_t* cand_i;      // [n_cand][4]: node, capacity type (KP_CT_*), catalog row, template (-1)
    const int32_t* cand_off;    // [n_cand + 1] CSR into cand_pods
    const int32_t* cand_pods;   // reschedulable pods of each candidate
    const double* cand_price;   // [n_cand]
    const int64_t* cand_cap;    // [n_cand][R] capacity returned to the candidate's NodePool limits
    const int32_t* rank;        // [P] queue position of each pod (NewQueue order)
    const uint64_t* pend_bits;  // [PW] pending pods by queue position
    int32_t PW;
    const uint64_t* init_bits;  // [EW] StateNode.Initialized() by node
    int32_t n_pending;
    const int64_t* alloc_act;   // [n_active][astride] allocatable of the active axes (EvalEnv.alloc)
    int32_t astride;
    // per-worker scratch
    int32_t ring_cap;           // >= pods of any probe
    int32_t* ring;              // [workers][ring_cap] queue entries: pod | relaxed << 30 | pending << 31
    // preference relaxation (relax != 0, d.relax_next): an entry with the relaxed bit carries its class (| fresh << 31:
    // not yet offered to the existing nodes) and shape here; other entries use the pod's input class / shape
    int32_t relax;
    int32_t* ring_cls;          // [workers][ring_cap]
    int32_t* ring_shape;        // [workers][ring_cap]
    int32_t* ring_last;         // [workers][ring_cap] Queue.lastLen of the entry (-1: never pushed)
    int32_t* pnode;             // [workers][ring_cap] FULL variant: 0 = an existing node took the pod, -1 = none does
    int64_t* delta;             // [workers][n_active][E] requests added to node j by this probe (valid: mod bit)
    uint64_t* pbits;            // [workers][PW] probe pods by queue position (all zero between probes)
    int32_t* next_probe;        // [3] work counters: fast variant, full variant, probes handed to the full variant
    int32_t* retry;             // [n_probes] probes the fast variant handed over
    kp_probe_result* out;       // [n_probes]
    int64_t* stats;             // [CS_COUNT]
    // kp_consolidate_command's read-back of one REPLACE probe (FULL variant, one probe per launch), else null:
    // rec_i = {decision, template, spot-narrowed, n options, options in price order [64], held IDs}, the NodeClaim's
    // requirements digest after FinalizeScheduling (rec_hdr [K], rec_words [DW]) and its held reservation IDs
    int32_t* rec_i;
    ReqHdr* rec_hdr;
    uint64_t* rec_words;
    // topology (consolidate_kernel<..., TOPO>): per-worker probe counts (ProbeTopo, kp_eval.h) and the probes' starting
    // decrements — the value-keyed counts of the pods each probe reschedules, one row of 64 counts per group:
    // single-node probe c: rows [dec_soff[c], dec_soff[c + 1]); multi-node probe i: rows [dec_moff[i], dec_moff[i + 1])
    int32_t G, HG;
    int32_t* pt_cnt;            // [workers][G][64]
    uint64_t* pt_known;         // [workers][G]
    int32_t* pt_hd;             // [workers][HG][E + 1]
    const uint64_t* pt_dgk;     // [G]
    const int32_t* dec_soff;
    const int32_t* dec_moff;
    const int32_t* dec_g;       // [rows] group of the row
    const int32_t* dec_v;       // [rows][64]
    // hostname pod affinity (a self-selecting pod bootstraps a domain only when no hostname domain holds a selected
    // pod): per probe, the positive-domain count of each such group after its candidates' pods come off —
    // hpos0[(single ? candidate : n_cand + prefix) * n_ha + ga]; tg_ha[g] = ga or -1
    // late topology identities (KpDev.tg_late) each probe's NewTopology creates: single-node probe ci / multi-node
    // probe i (null: none)
    const uint64_t* born_s;
    const uint64_t* born_m;
    int32_t n_ha;
    const int32_t* hpos0;
    const int32_t* tg_ha;
    // chunk headroom summary: cmax0[w][ai] = the largest headroom on active axis ai over the nodes of 64-node chunk w
    // (kp_launch_cons_chunk_max, after the existing-node tables); each probe copies it to LDS and lowers a chunk's entry
    // to its true maximum whenever it has the chunk's headroom in hand, so the entries stay upper bounds and a pod whose
    // request exceeds one on some axis skips the chunk without loading it (use_cmax: the LDS plan has room)
    const int64_t* cmax0;       // [EW][KP_LDS_AXES]
    int32_t use_cmax;
    // multi-node probes' pods (multi_union_kernel): [ulen] {pod | pending << 31, candidate or -1}, in queue order; null:
    // every probe marks and scans its own queue-position bitmap
    const int2* ulist;
    const int32_t* ulen;
    int32_t profile;            // s_memtime stage cycles (KPSIM_PROFILE)
    int64_t* prof_probe;        // KPSIM_PROFILE: [n_probes][4] cycles of build, existing-node placement, total; pods
    int32_t no_fast;            // diagnostics: every probe on the FULL variant (KPSIM_CONS_NOFAST)
    // MUT (ExistingNode.Add's requirement merge changes nodes, kp_solve_prepare's mutators): a probe that reschedules a
    // mutator's pod (mut_s[candidate] / mut_m[prefix]) runs on the FULL variant's MUT instantiation, serially over its
    // queue; a node whose requirements its merges change gets a copy of its digest (slot ov_slot[j], valid while the
    // probe's LDS bit mutn[j] is set), and class × node compatibility of such a node is evaluated against the copy
    int32_t mut;                // some probe of the pass is a MUT probe
    const int32_t* mut_s;       // [n_cand]
    const int32_t* mut_m;       // [multi-node probes]
    int32_t ov_cap;             // digest copies per worker
    int32_t* ov_slot;           // [FULL workers][E]
    ReqHdr* ov_hdr;             // [FULL workers][ov_cap][K]
    uint64_t* ov_words;         // [FULL workers][ov_cap][DW]
    // dynamic LDS plan (kp_cons_plan_lds)
    int32_t n_store;            // chunks in the fast variant's LDS headroom store (kp_cons_plan_lds)
    int32_t off_hdr, off_words, off_rem, off_excl, off_mod, off_init, off_xtc, off_touch, off_hmod, off_cmax, off_hs, off_hpos;
    int32_t off_mutn, off_rcap;
    int32_t lds_bytes;
};
