// kp_layout.h — device-resident table layout shared by the host encoder (kp_host.cpp) and the gfx950
// kernels (kp_kernels.hip).  Everything here is plain data: the host fills a KpDev of device pointers
// and passes it by value to every kernel.
//
// Encoding:
//   * label requirement sets (scheduling.Requirements) become DIGESTS: per solve key k a header
//     {flags, minValues, gt, lt} plus a value bitset of nw[k] u64 words over that key's value dictionary
//     (catalog values first, then values that only appear in pod/NodePool requirements);
//   * the catalog's single-valued labels become u16 value ids per (key, type); multi-valued labels
//     (zone, capacity-type, zone-id, reservation-*) become a u64 value mask per (key, type);
//   * offerings become one u64 per type: bit (zone slot × capacity-type slot) set when an on-demand/spot
//     offering in that pool is Available (offering.go:148);
//   * instance-type option sets are bitsets of TW = ceil(T/64) words.
#pragma once
#include <stdint.h>

#ifndef KP_MAX_TYPES
#define KP_MAX_TYPES 2048            // TW <= 32
#endif
#define KP_TW_MAX (KP_MAX_TYPES / 64)
#define KP_DNE_TW 16                 // DoesNotExist-type words of a class key kept in the class cache (LDS); the words of
                                     // larger catalogs are read from HBM (dne_mask)
#define KP_MAX_NC 65535              // in-flight NodeClaims per solve (u16 ids in the LDS slice arrays)
#define KP_NC_FIRST 4096             // slice capacity a solve is first planned with (kp_solve grows it on overflow)
#define KP_MAX_KEYS 96               // label keys per solve
#define KP_MAX_CLASS_KEYS 32         // label keys constrained by one pod class / template
#define KP_MAX_SLOTS 64              // zone slots × capacity-type slots
#define KP_MAX_NP 63                 // NodePools (templates) per solve: template bitmasks are u64, bit 63 a flag
#define KP_MAX_R 16                  // resource axes
#ifndef KP_NWAVES
#define KP_NWAVES 8                  // waves in the single-workgroup FFD kernel (kp_ffd_*_topo.hip: KP_NWAVES_TOPO)
#endif
#ifndef KP_NWAVES_TOPO
#define KP_NWAVES_TOPO 4             // waves of the topology instantiations
#endif
// the FFD headers' namespace per wave count (kp_w8, kp_w4): one definition per name across the kp_ffd_*.hip units
#define KP_WNS_CAT2(n) kp_w##n
#define KP_WNS_CAT(n) KP_WNS_CAT2(n)
#define KP_WNS KP_WNS_CAT(KP_NWAVES)
#define KP_LDS_AXES 6                // allocatable axes staged in LDS
#define KP_MAX_SCR_WORDS 64          // value-bitset words of one class's keys (per-wave LDS scratch)
#define KP_MAX_MIN_WORDS 64          // value bitset for a minValues distinct count (4096 values)
#define KP_LDS_BYTES (160 * 1024)    // LDS per workgroup on gfx950
#ifndef KP_MAX_TOPO
#define KP_MAX_TOPO 32               // topology groups constraining one pod class
#endif
#ifndef KP_MAX_TOPO_REC
#define KP_MAX_TOPO_REC 64           // ... recording (counting) its pods
#endif
#define KP_SNAP_ROWS 8               // constraining groups the FFD kernel snapshots / prefilters per pod (LDS)
#define KP_CC_REC 16                 // recording groups a ClassCache holds (the rest are read from cls_tr)
#define KP_CC_TC 16                  // constraining groups a ClassCache holds (the rest are read from cls_tc)
#define KP_MAX_TOPO_KEYS 8           // distinct value-keyed topology keys among a class's constraining groups
#define KP_TRACE_N 16384             // diagnostics ring (KPSIM_TRACE_*)           // topology groups recording one pod class's placements

// cls_flags bits
#define CF_OFFERING 1u               // constrains an offering key
#define CF_MINV 2u                   // carries minValues
#define CF_NOKEYS 4u                 // no requirement keys
#define CF_TOPO 8u                   // topology: constrained by or recorded into some group (never quick-accepted)
#define CF_TOPO_CONS 16u             // constrained by some group (AddRequirements runs in NodeClaim.Add)
#define CF_TOPO_QREC 32u             // every recording group's node filter is decidable from a NodeClaim's template
                                     // alone (no node-affinity filter owned by another class): quick accepts record

// tg_info.x
#define TG_TYPE 3                    // KP_TOPO_SPREAD / AFFINITY / ANTI_AFFINITY
#define TG_INVERSE 4
#define TG_HOST 8

// ReqHdr.flags
#define RF_DEF 1u                    // key present in the Requirements map
#define RF_CMP 2u                    // complement
#define RF_GT 4u
#define RF_LT 8u
#define RF_MIN 16u

// per solve key flags (KpDev.kflags)
#define KF_WELL_KNOWN 1u             // AllowUndefinedWellKnownLabels
#define KF_CAT_SINGLE 2u             // catalog label key, every type has <= 1 value
#define KF_CAT_MULTI 4u              // catalog label key with a multi-valued type (zone, capacity-type, ...)
#define KF_RESV_ROWS 8u              // the reservation-id label beyond 64 values: a type's values are its ResvTab rows' IDs

// type value ids for single-valued keys
#define VAL_DNE 0xFFFFu              // label DoesNotExist on the type
#define VAL_ABSENT 0xFFFEu           // key absent from the type's Requirements map (never checked)

struct ReqHdr {
    uint32_t flags;
    int32_t minv;
    int64_t gt;
    int64_t lt;
};

// Reserved offerings of the catalog (offering.go:164-194: one per capacity reservation of the EC2NodeClass), SoA in
// HBM (the FFD kernel stages small tables in LDS).  Rows are ordered by instance type and placed so that a type's
// rows lie inside one 64-row word (padding rows: type -1, unavailable); type_ro[t] packs that word and the rows' span.
// rid is the row's reservation (a dense index < nrid: its ReservationManager slot and its bit in a NodeClaim's held
// set of ridw words); ridv / zone / zid / rtype are value ids of the offering-role keys (zid, rtype -1: none).
#define KP_MAX_RO 1024               // reserved-offering rows (incl. padding) per catalog
#define KP_RO_W (KP_MAX_RO / 64)     // words of a row bitset or a held-reservation set
#define KP_RO_STAGE 128              // FFD kernel: tables of up to this many rows are staged in LDS
struct ResvTab {
    int32_t n, ctv, nrid, w;         // rows, capacity-type value id of "reserved", reservation IDs, row words
    int32_t ridw, pad;               // words of a held set: ceil(nrid / 64)
    const int32_t* type;             // [n] instance type row (-1: padding)
    const int32_t* zone;
    const int32_t* zid;
    const int32_t* rid;
    const int32_t* ridv;
    const int32_t* rtype;
    const uint64_t* avail;           // [w] bit i of word i / 64: row i is Available
    const int32_t* rid_vid;          // [nrid] reservation-id value id of reservation r
};
// type_ro[t] = word << 16 | first bit << 8 | rows: the type's reserved-offering rows within their word (0: none)

// Static operands of one (class, constraining topology group) entry, so the FFD kernel's per-pod prefilter setup reads
// one row instead of walking cls_tc → tg_info → the class digest: flags = type | self << 2 | hostname << 3; key = the
// group's key, or -1 - its row of tg_hcnt for a hostname group; podhas = the class's domains of the key (value ids < 64
// its requirement admits), vmask = the key's dictionary (value ids < nval).
// A self-selecting hostname pod affinity whose pod requirements restrict the hostname (podDomains In / NotIn a list):
// hdom = (n << 2) | 1 (In) or 2 (NotIn), podhas = the offset of the list's n existing nodes in KpDev.tce_hosts; hdom = 0
// when podDomains holds every host.
struct KpTopoCons {
    int32_t g, key, flags, skew, mindom, hdom;
    uint64_t podhas, vmask;
};
// ... of one (class, recording topology group) entry: flags = type | inverse << 2 | hostname << 3; key as above;
// skip = the templates on which TopologyNodeFilter's taint policy leaves the placement uncounted (a spread group with
// nodeTaintsPolicy Honor whose owner does not tolerate the template).
struct KpTopoRec {
    int32_t g, key, flags, late;  // late: the group's late-identity bit or -1 (KpDev.tg_late)
    uint64_t skip;
};

// Device pointers and sizes for one solve (catalog tables + solve tables + state + outputs).
struct KpDev {
    // ---------------- catalog (uploaded once per epoch) ----------------
    int32_t T, TW, R, K;             // types, option words, resource axes, solve keys
    int32_t n_slots;                 // zone × capacity-type slots
    int32_t n_multi;                 // multi-valued catalog keys
    const uint16_t* type_val;        // [K_cat][T] (indexed by kcat[k])
    const uint64_t* multi_mask;      // [n_multi][T]
    const uint16_t* multi16;         // [n_multi][T] same masks as u16 when every multi key has <= 16 catalog values, else null
    const uint64_t* dne_mask;        // [K_cat][TW] types whose label is DoesNotExist (or an empty In)
    const int64_t* alloc;            // [R][T]
    const int64_t* cap;              // [R][T]
    const uint64_t* avail_zc;        // [T] available od/spot offerings by slot
    const double* slot_price;        // [T][KP_MAX_SLOTS] price of the (type, slot) offering
    const int32_t* slot_zone;        // [n_slots] zone value id
    const int32_t* slot_ct;          // [n_slots] capacity-type value id
    const int32_t* slot_zoneid;      // [n_slots] zone-id value id or -1 (offering has no zone-id)
    const uint32_t* name_rank;       // [T] rank of the type name (OrderByPrice tie-break)
    const uint64_t* nonneg;          // [TW] types whose allocatable is non-negative everywhere

    // ---------------- solve keys ----------------
    const uint32_t* kflags;          // [K]
    const int32_t* kcat;             // [K] catalog key index or -1
    const int32_t* kmulti;           // [K] multi index or -1
    const int32_t* woff;             // [K] word offset in a digest
    const int32_t* nw;               // [K] words
    const int32_t* nval;             // [K] dictionary size
    const int32_t* vbase;            // [K] offset into val_isint/val_int
    const uint8_t* val_isint;        // strconv.Atoi succeeded
    const int64_t* val_int;
    int32_t DW;                      // digest words
    int32_t key_zone, key_ct, key_zoneid, key_resvid, key_resvtype;  // offering-key roles (-1 absent)

    // ---------------- classes (pod classes, then one pseudo-class per template) ----------------
    int32_t C;                       // pod classes
    int32_t NT;                      // templates (NodePools in weight order)
    const int32_t* cls_koff;         // [C+NT+1] CSR into cls_keys
    const int32_t* cls_keys;         // solve key ids constrained by the class
    const int32_t* cls_wsoff;        // parallel to cls_keys: word offset of the key in the wave scratch
    const ReqHdr* cls_hdr;           // [C+NT][K]
    const uint64_t* cls_words;       // [C+NT][DW]
    const uint32_t* cls_flags;       // [C+NT] bit0: defines an offering key, bit1: has minValues, bit2: no keys
    uint64_t* V;                     // [C+NT][TW] per-class single-valued label compatibility (class_mask kernel)

    // ---------------- templates ----------------
    const uint64_t* tmpl_rows;       // [NT][TW] GetInstanceTypes(nodepool) rows
    uint64_t* tmpl_opts;             // [NT][TW] NodeClaimTemplate.InstanceTypeOptions (template_init kernel)
    int32_t* tmpl_ok;                // [NT]
    const uint64_t* tol;             // [C] bit j: class tolerates template j's taints (templates <= KP_MAX_NP)
    const int64_t* daemon;           // [NT][R]
    const uint8_t* limit_set;        // [NT][R]
    int64_t* remaining;              // [NT][R] (mutated by the FFD kernel)
    uint64_t* tmpl_lmask;            // [NT][TW] types within each template's remaining limits (FFD kernel scratch)
    const int32_t* min_keys;         // [NT][KP_MAX_CLASS_KEYS] keys carrying minValues (-1 terminated)

    // ---------------- pods ----------------
    int32_t P;
    int32_t* pod_cls;                // [P] (rewritten by the FFD kernel when a pod relaxes)
    int32_t* pod_shape;              // [P] id of (class, requests)
    // preference relaxation (kp_host.cpp expand_preferences); relax_next == nullptr: no class can relax
    const int32_t* relax_next;       // [C] the class after one preferences.Relax step, -1 when none is left
    const int32_t* shape_next;       // [shapes] the shape of (relax_next[class], same requests)
    const int32_t* pod_cls0;         // [P] input classes / shapes, restored into pod_cls / pod_shape per execute
    const int32_t* pod_shape0;
    int32_t* last_ep;                // [P] epoch of last_len (Queue.Push(pod, relaxed) clears lastLen: a new epoch)
    int32_t best_effort;             // MIN_VALUES_POLICY=BestEffort: unmet minValues relax instead of failing
    const int64_t* pod_req;          // [P][R]
    const int32_t* queue0;           // [P] queue order (NewQueue sort), device-sorted
    int32_t active_axes[KP_MAX_R];   // axes any pod/daemon requests, LDS-staged first
    int32_t n_active;

    // ---------------- state ----------------
    int32_t NCcap;
    ReqHdr* nc_hdr;                  // [NCcap][K]
    uint64_t* nc_words;              // [NCcap][DW]
    uint64_t* nc_opts;               // [NCcap][TW]
    int64_t* nc_req;                 // [NCcap][R]
    int32_t* nc_tmpl;                // [NCcap]
    const ReqHdr* empty_hdr;         // [K] all-undefined digest (template init)
    const uint64_t* empty_words;     // [DW]
    int32_t* qbuf;                   // [P] queue ring
    int32_t* last_len;               // [P]

    // ---------------- outputs ----------------
    int32_t* pod_result;             // [P]
    int32_t* pod_order;              // [P]
    int32_t* nc_count;               // [1]
    int32_t* nc_npods;               // [NCcap]
    int32_t* nc_slice_pos;           // [NCcap]
    int32_t* nc_nopts;               // [NCcap]
    int32_t* nc_valid;               // [NCcap]
    int32_t M;                       // max instance types (Truncate)
    int32_t* nc_types;               // [NCcap][M]
    int32_t* nc_ntypes;              // [NCcap]
    int64_t* stats;                  // [16]
    int32_t* err;                    // [1] device-side error code (capacity overflow etc.)
    int32_t profile;                 // accumulate per-stage evaluation cycles (diagnostics)
    int32_t topo_cands;              // NodeClaims evaluated per block round for a topology pod (<= KP_NWAVES)
    int32_t team_eval;               // topology pods: one candidate at a time, evaluated by the whole block (eval_wave TEAM)
    int32_t noop_quick;              // fast loop: quick accept on a NodeClaim whose merge with the class changes nothing
    int32_t team_first;              // slow path: a first candidate that needs the full Add is evaluated by the whole block
    int32_t block_sort;              // slow path: the commit's slice move by the whole block (block_sort_move)
    int32_t trace_pod;               // diagnostics (KPSIM_TRACE_POD): the slow path logs this pod's evaluations
    int32_t trace_max;               //   KPSIM_TRACE_CLASS: only pods with index <= KPSIM_TRACE_MAXPOD
    int32_t* trace;                  //   [1 + 6 * KP_TRACE_N]: count, then {round, nodeclaim (-1-j: template j), ok, flags, held lo/hi}

    // ---------------- existing nodes (ExistingNode, [core] scheduling/existingnode.go) ----------------
    int32_t E, EW;                   // existing nodes in scheduling order; words of an E-bit row
    const ReqHdr* ex_hdr0;           // [E][K] NewLabelRequirements(node labels) + hostname In [name]
    const uint64_t* ex_words0;       // [E][DW]
    ReqHdr* ex_hdr;                  // [E][K] working copy (ExistingNode.Add narrows requirements)
    uint64_t* ex_words;              // [E][DW]
    const int64_t* ex_avail;         // [E][R] StateNode.Available()
    const int64_t* ex_req;           // [E][R] remaining daemonset requests (initial ExistingNode.requests)
    int64_t* ex_head;                // [n_active][E] available - requests on the active axes (working)
    uint8_t* ex_static;              // [E] Fits holds on every inactive axis and no available quantity is negative
    uint64_t* XT;                    // [C][EW] taints tolerated ∧ static fit ∧ Requirements.Compatible(node, class)
    const uint64_t* ex_tol;          // [C][EW] the class tolerates the node's taints
    const int32_t* cls_xkoff;        // [C+NT+F+1] CSR of every key a digest row constrains (incl. hostname): pod
                                     // classes, templates (empty), then the F spread node-filter rows (tg_frow)
    const int32_t* cls_xkeys;
    int32_t ex_mayfix;               // some class has a NotIn/DoesNotExist key: Add may change node requirements

    // ---------------- topology ([core] scheduling/topology.go, topologygroup.go) ----------------
    // One group per (pod class, topology term) plus one inverse group per required anti-affinity term.  Value-keyed
    // groups (zone, capacity-type, ... : <= 64 dictionary values) count per value id; hostname groups count per host
    // domain h = existing node j, or E + n for in-flight NodeClaim n.  Counts only grow during a Solve.
    int32_t G;                       // groups
    int32_t HN;                      // hostname-count row length (E + NCcap)
    int32_t key_host;                // kubernetes.io/hostname solve key or -1
    const int4* tg_info;             // [G] {type | inverse << 2 | hostname << 3, key, max_skew, min_domains (0 nil)}
    const int32_t* tg_hrow;          // [G] row of tg_hcnt (hostname groups), else -1
    const int32_t* tg_owner;         // [G] class owning the term (spread node filter)
    const int32_t* tg_pol;           // [G] spread node filter: bit0 nodeAffinityPolicy Honor, bit1 nodeTaintsPolicy Honor
    const int2* tg_frow;             // [G] bit0 of tg_pol: the filter's digest rows [x, x + y) of cls_hdr / cls_xkoff
    // groups that Topology.Update creates when a pod relaxes into a spec owning them (kp_host.cpp topo_build): bit of
    // the group's late identity or -1 (null: none); cls_birth[c] = late identities class c owns (a pod relaxing into c
    // creates them); born0 = those a pod of the Solve owns from the start.  Records skip a late group until it is born.
    int32_t snap_rows;               // TopoSnap rows in the FFD kernel's LDS plan (SnapRow)
    const int32_t* tg_late;
    const uint64_t* cls_birth;
    uint64_t born0;
    // variant groups (an identity only relaxed pods create, its owners' node filters / minDomains differing): per late
    // bit, the bits of its identity's variants (itself alone for a plain late group) and its group; null without
    // variants.  A relaxation births a variant only while none of its siblings is born (topo_birth), and a class's
    // constraint entry on a variant routes to the born sibling (fill_class_cache, topo_prefilter_setup).
    const uint64_t* late_sib;
    const int32_t* late_grp;
    int32_t* tg_cnt;                 // [G][64] counts by value id (value-keyed groups)
    uint64_t* tg_known;              // [G] value ids present in the group's domains map
    int32_t* tg_hcnt;                // [hostname groups][HN]
    int32_t* tg_pos;                 // [G] hostname domains with a positive count (affinity bootstrap)
    const int32_t* cls_tcoff;        // [C+1] CSR: groups that constrain the class (owned forward, selecting inverse)
    const int32_t* cls_tc;           //   entry: group | self-selecting << 30
    const int32_t* cls_troff;        // [C+1] CSR: groups that record the class's placements
    const int32_t* cls_tr;
    const uint8_t* cls_kneutral;     // parallel to cls_keys: 1 = key added only so topology can narrow it
    const uint8_t* vrank;            // [K][64] rank of value id v among the key's values by name (tie-break)
    const struct KpTopoCons* cls_tce; // parallel to cls_tc: the entry's static operands (FFD kernel prefilter setup)
    const int2* tce_hosts;           // KpTopoCons.hdom lists: (existing node, 1 = it still holds a selected pod once its
                                     // own consolidation candidate's pods leave)
    const struct KpTopoRec* cls_tre;  // parallel to cls_tr: the entry's static operands (topology quick accept's Record)

    // ---------------- FFD kernel LDS plan (kp_ffd_plan_lds) ----------------
    // Dynamic LDS after the fixed FfdShared block: slice arrays sized by lds_ncmax, the staged type tables
    // sized by lds_tpad, and the quick-accept headroom table hr[lds_A][lds_nq].
    int32_t lds_ncmax;               // in-flight NodeClaim capacity of the kernel (<= KP_MAX_NC, <= NCcap)
    int32_t slice_hbm;               // the slice arrays are in HBM (g_key ...): more NodeClaims than LDS holds
    uint32_t* g_key;                 // [NCcap] HBM slice arrays (allocated for plans above KP_NC_FIRST)
    uint16_t* g_ord;
    uint16_t* g_last;
    uint8_t* g_tmpl;
    int32_t lds_tpad;                // staged-table row stride (T rounded up to 64)
    int32_t lds_nstage;              // allocatable axes staged in LDS
    int32_t lds_A;                   // quick-accept axes (= n_active when n_active <= KP_LDS_AXES, else 0)
    int32_t lds_nq;                  // NodeClaims with a quick-accept headroom row (ids < lds_nq)
    int32_t alloc_global;            // large slice plans: allocatable read from alloc_act in HBM, not staged in LDS
    const int64_t* alloc_act;        // [lds_nstage][lds_tpad] allocatable of the staged axes (alloc_global)
    int32_t off_key, off_ord, off_last, off_tmpl, off_alloc, off_avail, off_multi, off_ro, off_tsnap, off_hr, off_qw;
    int32_t lds_bytes;
    int32_t qshift[KP_LDS_AXES];     // headroom scale per quick axis: value >> qshift fits 30 bits

    // ---------------- reserved capacity ([core] scheduling/reservationmanager.go, nodeclaim.go) ----------------
    const ResvTab* ro;               // reserved offerings (device copy of the header; null: none)
    const uint32_t* type_ro;         // [T] the type's rows (ro_span_bits), see ResvTab
    const double* ro_price;          // [ro_n] price of row i
    int32_t ro_n, ro_w, ro_nrid, ro_ridw;  // the header's sizes, for kernels that size loops without reading it
    int32_t ro_stage;                // FFD kernel: the rows fit its LDS plan and are staged there
    int32_t resv_on;                 // ReservedCapacity gate ∧ reserved offerings exist: NodeClaim.Add reserves
    const int32_t* rcap0;            // [ro_nrid] ReservationManager capacity per reservation (least over its offerings)
    uint64_t* nc_held;               // [NCcap][ro_ridw] reservations a NodeClaim holds (NodeClaim.reservedOfferings' IDs)
    int32_t* nc_rlive;               // [NCcap] the NodeClaim's options keep a compatible available reserved offering

    // a device copy of this struct (uploaded before each FFD launch): out-of-line device functions take it instead of
    // the kernel argument, whose address would otherwise escape and put every field read of the kernel in scratch
    const KpDev* self;
};

// stats slots
enum {
    ST_POPPED = 0, ST_NC_EVALS, ST_NC_SCANNED, ST_TMPL_EVALS, ST_EXIST_EVALS, ST_SORT_FAST, ST_SORT_FULL,
    ST_MEMO_SKIPS, ST_CYC_POP, ST_CYC_SORT, ST_CYC_SCAN, ST_CYC_TMPL, ST_CYC_COMMIT, ST_CYC_SORT_FULL,
    ST_EV_REQ = 16, ST_EV_MASK, ST_EV_OFF, ST_EV_TYPES, ST_EV_MIN, ST_EV_CALLS,
    ST_QUICK = 24, ST_SLOW, ST_WITNESS_MISS, ST_CYC_QPOP, ST_CYC_QSCAN, ST_CYC_QCHECK, ST_CYC_QCOMMIT,
    ST_N_NOINV = 32, ST_N_WINMOVE, ST_N_LDSSORT, ST_N_PIVOT, ST_N_WINLOAD, ST_N_FLUSH, ST_N_SHAPE, ST_EXIST_PLACED = 44,
    ST_TOPO_QUICK = 45, ST_CYC_TSETUP, ST_CYC_TSCAN,
    // KPSIM_PROFILE: why evaluations fail (requirement merge, topology narrowing, no type left, minValues, other)
    ST_REJ_REQ = 48, ST_REJ_TOPO, ST_REJ_TYPES, ST_REJ_MIN,
    // KPSIM_PROFILE: topology pods past the prefilter — no surviving NodeClaim, class records through another class's
    // node filter (not QREC), NodeClaim without a quick row, class not absorbed, quick row present; witness fits
    ST_TQ_WHY = 52, ST_SLOW_WHY = 59,
    // KPSIM_PROFILE: one outer iteration of the solve loop cut into segments (thread 0's clock): the fast loop and the
    // barrier that opens the slow path; the topology section (existing nodes, prefilter, scan, topology quick accept);
    // the class cache fill; the candidate evaluations; commit / templates / slice move / closing barrier; then the
    // iterations that end in a topology quick accept (count, cycles from the slow path's start to their end)
    ST_SEG = 70, ST_TQ_ITERS = 75, ST_TQ_CYC = 76, ST_COUNT = 80
};
