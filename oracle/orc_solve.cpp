// ORACLE — test infrastructure only (see oracle/README.md). Never linked into libkpsim; only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg load liboracle.so, and only as the checker.
//
// CPU restatement of the reference's provisioning scheduling simulation:
//   [core] pkg/controllers/provisioning/scheduling/scheduler.go  NewScheduler / Solve / add
//          (sort.Slice(newNodeClaims, by len(Pods)) before every in-flight attempt, templates in weight order,
//           filterByRemainingResources / subtractMax NodePool limits)
//   [core] .../scheduling/queue.go          NewQueue (byCPUAndMemoryDescending), Pop, Push
//   [core] .../scheduling/nodeclaim.go      NewNodeClaim, Add, FinalizeScheduling,
//                                            filterInstanceTypesByRequirements (compatible, fits, hasOffering, minValues)
//   [core] .../scheduling/existingnode.go   ExistingNode.Add
//   [core] pkg/cloudprovider/types.go       InstanceTypes.OrderByPrice / Truncate / SatisfiesMinValues,
//                                            Offerings.Available / Compatible / Cheapest
//   [core] pkg/utils/resources              Fits, Merge, MaxResources
// Core is sigs.k8s.io/karpenter v1.6.1-0.20250908174930-91341612ebc6 (reference go.mod:49), not vendored:
// semantics are recalled and pinned by the KATs from the reference's own suites
// (tests/golden/kats.json; pkg/providers/instancetype/suite_test.go:395-995).  In-tree inputs follow
// pkg/providers/instancetype/offering/offering.go:103-196 (offering requirements) and
// pkg/providers/instance/instance.go:62,293 (maxInstanceTypes = 60, Truncate).
#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../include/kpsim.h"
#include "gosort.h"
#include "orc_api.h"
#include "orc_req.h"

namespace orc {

struct Offering {
    Reqs reqs;
    double price = 0;
    bool available = false;
    int rid = -1;  // reserved offerings: dense index of the reservation ID (Solver::rid_names)
};

struct InstanceType {
    std::string name;
    Reqs reqs;
    std::vector<int64_t> cap, alloc;
    std::vector<Offering> offerings;
};

struct Taint {
    std::string key, value, effect;
};
struct Toleration {
    std::string key;
    int op = 0;
    std::string value, effect;
};

// k8s.io/api/core/v1 Toleration.ToleratesTaint
static bool tolerates_taint(const Toleration& t, const Taint& taint) {
    if (!t.effect.empty() && t.effect != taint.effect) return false;
    if (!t.key.empty() && t.key != taint.key) return false;
    if (t.op == KP_TOL_EXISTS) return true;
    return t.value == taint.value;
}
// [core] scheduling.Taints.ToleratesPod: every taint must be tolerated by some toleration
static bool tolerates_all(const std::vector<Taint>& taints, const std::vector<Toleration>& tols) {
    for (auto& taint : taints) {
        bool ok = false;
        for (auto& t : tols) ok = ok || tolerates_taint(t, taint);
        if (!ok) return false;
    }
    return true;
}

// [core] resources.Fits(candidate, total)
static bool fits(const std::vector<int64_t>& candidate, const std::vector<int64_t>& total) {
    for (int64_t q : total)
        if (q < 0) return false;
    for (size_t r = 0; r < candidate.size(); r++)
        if (candidate[r] > total[r]) return false;
    return true;
}

// metav1.LabelSelector over pod labels (labels.Selector semantics: In / NotIn / Exists / DoesNotExist)
struct LabelSel {
    bool nil = false;  // a nil selector selects nothing
    struct Term {
        std::string key;
        int op = 0;
        std::vector<std::string> values;
    };
    std::vector<Term> terms;
    bool matches(const std::map<std::string, std::string>& labels) const {
        if (nil) return false;
        for (auto& t : terms) {
            auto it = labels.find(t.key);
            const bool present = it != labels.end();
            const bool in = present && std::find(t.values.begin(), t.values.end(), it->second) != t.values.end();
            if (t.op == KP_OP_IN && !in) return false;
            if (t.op == KP_OP_NOT_IN && in) return false;
            if (t.op == KP_OP_EXISTS && !present) return false;
            if (t.op == KP_OP_DOES_NOT_EXIST && present) return false;
        }
        return true;
    }
};

// One topology term of a pod class (kp_topology_term)
struct TopoTerm {
    int type = 0, key = -1, max_skew = 1, min_domains = -1, aff_pol = KP_POLICY_HONOR, taint_pol = KP_POLICY_IGNORE;
    bool preferred = false;  // ScheduleAnyway spread / weighted (anti-)affinity: no inverse group (only required terms)
    LabelSel sel;
    std::vector<std::string> namespaces;
};

struct PodClass {
    Reqs reqs;
    // MakeTopologyNodeFilter's requirements: the nodeSelector with each remaining required node-affinity term (ORed),
    // no preference; and NewStrictPodRequirements (podDomains in AddRequirements) when a preferred term is in reqs
    std::vector<Reqs> filter;
    Reqs strict;
    bool has_strict = false;
    std::vector<Toleration> tols;
    std::string ns = "default";
    std::map<std::string, std::string> labels;
    std::vector<TopoTerm> terms;
};

// [core] scheduling/topologygroup.go TopologyGroup.  One group per (pod class, term); Go keeps one TopologyGroup per
// Hash() (Topology.Update: topologyGroups[hash], first insert wins), so every group of one identity takes the first
// owner's selector, minDomains, node filter and tolerations (Solver::adopt) and they all count the same pods.
// `cnt` is the domains map (domain value id → count; emptyDomains = the domains with count 0, since counts only grow
// within a Solve).  Hostname groups know every registered host implicitly (NewNodeClaim and NewExistingNode
// Register their hostnames in every hostname group), so only recorded hosts are stored.
struct TopoGroup {
    int type = 0, key = -1;
    int late = -1;             // late identity bit (build_topology): created by Topology.Update when a pod relaxes
    bool host = false;
    bool inverse = false;      // inverseTopologyGroups (updateInverseAntiAffinity): constrains the pods it selects
    int owner = -1;            // class that owns the term
    int ident = -1;            // TopologyGroup.Hash() identity (build_topology)
    int sem = -1;              // class whose TopologyGroup the identity keeps (its first owner): node filter, tolerations
    int max_skew = 0, min_domains = -1;
    int aff_pol = KP_POLICY_IGNORE, taint_pol = KP_POLICY_IGNORE;  // TopologyNodeFilter (spread only)
    std::vector<uint8_t> sel;  // per class: selects(pod) = namespace ∈ namespaces ∧ selector matches labels
    std::map<int, int> cnt;
};
struct Pod {
    int cls = 0;
    std::vector<int64_t> req;
    int64_t ts = 0;
    std::string uid;
};

struct Template {
    int np_index = 0;
    std::string name;
    int weight = 0;
    Reqs reqs;
    std::vector<Taint> taints;
    std::vector<int64_t> daemon;
    std::vector<uint8_t> limit_set;
    std::vector<int64_t> remaining;
    std::vector<int> options;  // InstanceTypeOptions (catalog rows, order = GetInstanceTypes order)
};

struct NodeClaim {
    int id = 0;
    int tmpl = 0;
    int host = 0;  // hostname-placeholder value id (negative)
    Reqs reqs;
    std::vector<int> options;
    std::vector<int64_t> requests;
    std::vector<int> pods;
    bool valid = true;
    std::vector<int> truncated;
    std::vector<int> held;  // reservedOfferings: reservation IDs this NodeClaim holds (sorted rid indices)
};

struct ExistingNode {
    Reqs reqs;
    std::vector<Taint> taints;
    std::vector<int64_t> available, requests;
    int host = 0;  // hostname value id
};

// A NodePool as buildDomainGroups sees it (every NodePool, also those whose options end up empty)
struct PoolDomains {
    Reqs reqs;
    std::vector<Taint> taints;
    std::vector<int> rows;
};

struct Result {
    std::vector<NodeClaim> ncs;  // creation order
    Dict D;
};

struct Solver {
    Dict& D;
    int R = 0;
    std::vector<InstanceType> own_types;
    const std::vector<InstanceType>* tp = &own_types;  // catalog rows (shared by consolidation probes)
    std::vector<Template> tmpls;
    std::vector<PodClass> own_classes;
    const std::vector<PodClass>* cp = &own_classes;
    std::vector<Pod> own_pods;
    const std::vector<Pod>* pp = &own_pods;
    std::vector<ExistingNode> own_existing;
    const std::vector<ExistingNode>* ex_base = &own_existing;  // state nodes (shared by consolidation probes)
    std::vector<int> ex_idx;                                 // existing nodes of this simulation, in order
    std::unordered_map<int, ExistingNode> ex_mod;            // copy-on-write: nodes that received pods
    std::vector<int> plist;           // pods of this simulation (indices into *pp); all per-pod state is by position
    std::vector<NodeClaim> ncs;       // creation order; nc.pods holds positions in plist
    std::vector<int> newNodeClaims;   // s.newNodeClaims slice (indices into ncs)
    std::vector<int> pod_result, pod_order;  // by position in plist
    int placements = 0;
    int hostname_key = -1;
    Req host_req;                     // hostname In [placeholder] of a new NodeClaim (no pod can select it)
    int next_host = 0;                // NewNodeClaim's hostname-placeholder counter (value id -2 - n)
    std::vector<TopoGroup> groups;    // Topology.topologyGroups ∪ inverseTopologyGroups
    std::vector<TopoGroup> groups_dg; // ... as buildDomainGroups left them, before countDomains
    std::vector<std::vector<int>> t_cons, t_rec;  // per class: groups that constrain / count its pods
    // TopologyGroup.Hash() identities that only a relaxed spec owns (see build_topology): per class, the late identities
    // it owns (a pod relaxing into the class creates them); born = those created so far in this simulation
    std::vector<uint64_t> cls_birth;
    int n_late = 0;
    uint64_t born = ~0ull;
    std::vector<std::vector<int>> ident_groups;  // identity → its (class, term) groups
    std::vector<int> late_ident;                 // late bit → identity
    std::vector<std::pair<int, int>> bound_pods; // (node, class) of the pods countDomains counts in this simulation
    std::vector<int> cls_origin;  // per class: its input class
    int n_input = 0;
    kp_solve_stats stats{};
    // ReservationManager ([core] scheduling/reservationmanager.go): capacity per reservation ID, the least
    // ReservationCapacity among the offerings that carry the ID; NodeClaims hold IDs (NodeClaim.reservedOfferings).
    std::vector<std::string> rid_names;
    std::vector<int> rcap;
    int resv_key = -1;         // karpenter.k8s.aws/capacity-reservation-id (cloudprovider.ReservationIDLabel)
    bool resv_on = false;      // ReservedCapacity feature gate ∧ the catalog has reserved offerings
    bool resv_strict = true;   // ReservedOfferingModeStrict (provisioning); Fallback in disruption simulations
    int trace_pod = getenv("ORC_TRACE_POD") ? atoi(getenv("ORC_TRACE_POD")) : -1;
    int trace_cls = getenv("ORC_TRACE_CLASS") ? atoi(getenv("ORC_TRACE_CLASS")) : -1;

    explicit Solver(Dict& d) : D(d) {}
    const InstanceType& ty(int t) const { return (*tp)[t]; }
    const Pod& pod_at(int li) const { return (*pp)[plist[li]]; }
    // the pod's class as preferences.Relax left it (a relaxed pod moves to its class's next relaxation stage)
    std::vector<int> pcls;            // by position in plist
    std::vector<int> relax_next;      // per class: the class after one Relax step, -1 when nothing is left to relax
    bool best_effort = false;         // MIN_VALUES_POLICY=BestEffort
    int cls_id(int li) const { return pcls.empty() ? pod_at(li).cls : pcls[li]; }
    const PodClass& cls_of(int li) const { return (*cp)[cls_id(li)]; }

    // compatible(it, reqs) = it.Requirements.Intersects(reqs) == nil
    bool compatible(const InstanceType& it, const Reqs& reqs) const { return reqs_intersects(D, it.reqs, reqs); }
    bool has_offering(const InstanceType& it, const Reqs& reqs) const {
        for (auto& o : it.offerings)
            if (o.available && reqs_compatible(D, reqs, o.reqs, true)) return true;
        return false;
    }
    // InstanceTypes.SatisfiesMinValues(requirements): minNeededInstanceTypes (the shortest prefix that satisfies every
    // minValues key) and whether the whole list satisfies them.
    bool satisfies_min_values(const std::vector<int>& its, const Reqs& reqs, int* min_needed = nullptr) const {
        if (min_needed) *min_needed = 0;
        if (!reqs.has_min_values()) return true;
        std::vector<std::pair<int, std::vector<int>>> seen;  // (key, sorted distinct values so far)
        for (auto& kv : reqs.m)
            if (kv.second.has_min) seen.push_back({kv.first, {}});
        for (size_t i = 0; i < its.size(); i++) {
            bool ok = true;
            for (auto& sk : seen) {
                Req r = ty(its[i]).reqs.get(sk.first);
                for (int v : r.values) sk.second.push_back(v);
                std::sort(sk.second.begin(), sk.second.end());
                sk.second.erase(std::unique(sk.second.begin(), sk.second.end()), sk.second.end());
                if ((int)sk.second.size() < reqs.m.at(sk.first).min_values) ok = false;
            }
            if (ok) {
                if (min_needed) *min_needed = (int)i + 1;
                return true;
            }
        }
        if (min_needed) *min_needed = (int)its.size();
        for (auto& sk : seen)
            if ((int)sk.second.size() < reqs.m.at(sk.first).min_values) return false;
        return true;
    }
    // filterInstanceTypesByRequirements.  MIN_VALUES_POLICY=Strict: a remaining list that fails SatisfiesMinValues is
    // emptied.  BestEffort: the list is kept and, when `relax` is given (NodeClaim.Add), every unsatisfied minValues
    // key is relaxed to the number of distinct values the list offers (SatisfiesMinValues' unsatisfiableKeys; the
    // NodeClaim's requirements carry the relaxed minValues from then on).
    std::vector<int> filter(const std::vector<int>& its, const Reqs& reqs, const std::vector<int64_t>& total,
                            Reqs* relax = nullptr) const {
        std::vector<int> out;
        for (int t : its) {
            const InstanceType& it = ty(t);
            if (compatible(it, reqs) && fits(total, it.alloc) && has_offering(it, reqs)) out.push_back(t);
        }
        if (reqs.has_min_values() && !satisfies_min_values(out, reqs)) {
            if (!best_effort) {
                out.clear();
            } else if (relax && !out.empty()) {
                for (auto& kv : relax->m) {
                    if (!kv.second.has_min) continue;
                    std::vector<int> vals;
                    for (int t : out)
                        for (int v : ty(t).reqs.get(kv.first).values) vals.push_back(v);
                    std::sort(vals.begin(), vals.end());
                    vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
                    if ((int)vals.size() < kv.second.min_values) kv.second.min_values = (int)vals.size();
                }
            }
        }
        return out;
    }

    // ------------------------------------------------------------------------------------------------
    // Topology ([core] scheduling/topology.go, topologygroup.go; recalled).  Go iterates maps when it
    // picks a domain among equal counts (nextDomainTopologySpread's `count < minCount`, nextDomainAffinity's first
    // match), so any tied domain is a valid Go outcome; this restatement (and the device) takes the smallest domain name.
    // ------------------------------------------------------------------------------------------------
    std::string dom_name(int key, int v) const {
        if (v >= 0) return D.vals[key][v];
        char b[48];
        snprintf(b, sizeof b, "hostname-placeholder-%04d", -2 - v);
        return b;
    }
    bool dom_less(int key, int a, int b) const { return dom_name(key, a) < dom_name(key, b); }
    static int count_of(const TopoGroup& g, int d, bool& known) {
        auto it = g.cnt.find(d);
        if (it != g.cnt.end()) {
            known = true;
            return it->second;
        }
        known = g.host;  // every registered host is a known (empty) domain
        return 0;
    }
    // domainMinCount(podDomains): hostname topologies have a min of 0; minDomains above the supported domain count → 0
    int64_t domain_min_count(const TopoGroup& g, const Req& podDom) const {
        if (g.host) return 0;
        int64_t mn = INT32_MAX;
        int num = 0;
        for (auto& kv : g.cnt)
            if (req_has(D, podDom, kv.first)) {
                num++;
                mn = std::min<int64_t>(mn, kv.second);
            }
        if (g.min_domains > 0 && num < g.min_domains) mn = 0;
        return mn;
    }
    // TopologyGroup.Get(pod, podDomains, nodeDomains) → the allowed domains (an In requirement; empty = DoesNotExist)
    Req topo_get(const TopoGroup& g, int cls, const Req& podDom, const Req& nodeDom) const {
        Req out;
        out.key = g.key;
        out.complement = false;
        // the domains examined: nodeDomains' values on the In path, else every known domain in nodeDomains.  (A
        // hostname nodeDomains is always In [the node's host]: NodeClaims and existing nodes carry hostname In [name].)
        std::vector<int> cand;
        const bool in_path = nodeDom.Operator() == OP_IN;
        if (in_path) {
            cand = nodeDom.values;
        } else {
            for (auto& kv : g.cnt)
                if (req_has(D, nodeDom, kv.first)) cand.push_back(kv.first);
        }
        if (g.type == KP_TOPO_SPREAD) {  // nextDomainTopologySpread
            const int64_t mn = domain_min_count(g, podDom);
            const int self = g.sel[cls];
            int best = 0;
            int64_t bc = INT32_MAX;
            bool found = false;
            for (int d : cand) {
                bool known;
                const int64_t c = (int64_t)count_of(g, d, known) + self;
                if (!known) continue;
                if (c - mn <= g.max_skew && (c < bc || (c == bc && found && dom_less(g.key, d, best)))) {
                    best = d;
                    bc = c;
                    found = true;
                }
            }
            if (found) out.values.push_back(best);
            return out;
        }
        if (g.type == KP_TOPO_ANTI_AFFINITY) {  // nextDomainAntiAffinity: empty domains the pod and node allow
            for (int d : cand) {
                bool known;
                const int c = count_of(g, d, known);
                if (known && c == 0 && req_has(D, podDom, d)) out.values.push_back(d);
            }
            std::sort(out.values.begin(), out.values.end());
            return out;
        }
        // nextDomainAffinity: domains the pod allows that hold a selected pod; a self-selecting pod with none
        // bootstraps a domain (first one compatible with the node domains, else any the pod allows)
        std::vector<int> known_doms;
        for (auto& kv : g.cnt) known_doms.push_back(kv.first);
        if (g.host && in_path)
            for (int d : nodeDom.values)
                if (!g.cnt.count(d)) known_doms.push_back(d);
        for (int d : known_doms) {
            bool k;
            if (count_of(g, d, k) > 0 && req_has(D, podDom, d)) out.values.push_back(d);
        }
        if (out.values.empty() && g.sel[cls]) {
            int pick = 0;
            bool found = false;
            for (int pass = 0; pass < 2 && !found; pass++)
                for (int d : known_doms)
                    if (req_has(D, podDom, d) && (pass == 1 || req_has(D, nodeDom, d)) &&
                        (!found || dom_less(g.key, d, pick))) {
                        pick = d;
                        found = true;
                    }
            if (found) out.values.push_back(pick);
        }
        std::sort(out.values.begin(), out.values.end());
        return out;
    }
    // Topology.AddRequirements + NodeClaim.Add's Compatible(nodeClaimRequirements, topologyRequirements) + Add:
    // every group that constrains the pod contributes its domains computed from the same nodeRequirements.
    bool topo_add(int li, Reqs& r, bool allow_wk) const {
        const int c = cls_id(li);
        if (t_cons.empty() || t_cons[c].empty()) return true;
        const PodClass& pc = (*cp)[c];
        Reqs topo = r;
        for (int gi : t_cons[c]) {
            const TopoGroup& g = groups[gi];
            // podDomains: the strict requirements' (no preferred term) requirement for the key; Exists without one
            const Req podDom = (pc.has_strict ? pc.strict : pc.reqs).get(g.key);
            const Req nodeDom = r.get(g.key);
            const Req dom = topo_get(g, c, podDom, nodeDom);
            if (dom.Len() == 0) return false;  // topologyError
            topo.add(D, dom);
        }
        if (!reqs_compatible(D, r, topo, allow_wk)) return false;
        r.add_all(D, topo);
        return true;
    }
    // TopologyNodeFilter.MatchesRequirements: Compatible with one of the filter's requirement sets
    bool filter_matches(const PodClass& fc, const Reqs& r, bool allow_wk) const {
        for (const Reqs& f : fc.filter)
            if (reqs_compatible(D, r, f, allow_wk)) return true;
        return false;
    }
    // Topology.Record(pod, taints, requirements): every group whose Counts(pod) holds records the domain(s) the pod
    // lands in; inverse groups owned by the pod record every value of the requirement.
    void topo_record(int li, const Reqs& r, const std::vector<Taint>& taints, bool allow_wk) {
        const int c = cls_id(li);
        if (t_rec.empty()) return;
        for (int gi : t_rec[c]) {
            TopoGroup& g = groups[gi];
            if (g.late >= 0 && !((born >> g.late) & 1ull)) continue;  // not created yet
            const Req dom = r.get(g.key);
            if (!g.inverse) {
                if (g.type == KP_TOPO_SPREAD) {  // TopologyNodeFilter.Matches
                    const PodClass& fc = (*cp)[g.sem];
                    if (g.aff_pol == KP_POLICY_HONOR && !filter_matches(fc, r, allow_wk)) continue;
                    if (g.taint_pol == KP_POLICY_HONOR && !tolerates_all(taints, fc.tols)) continue;
                }
                if (g.type != KP_TOPO_ANTI_AFFINITY) {  // the domain is recorded only once it is a single value
                    if (!dom.complement && dom.values.size() == 1) g.cnt[dom.values[0]]++;
                    continue;
                }
            }
            for (int v : dom.values) g.cnt[v]++;  // Values(): the excluded set of a complement
        }
    }

    bool nodeclaim_add(NodeClaim& nc, int li) {
        const Pod& pod = pod_at(li);
        const PodClass& pc = cls_of(li);
        const Template& tm = tmpls[nc.tmpl];
        if (!tolerates_all(tm.taints, pc.tols)) return false;
        Reqs r = nc.reqs;
        if (!reqs_compatible(D, r, pc.reqs, true)) return false;
        r.add_all(D, pc.reqs);
        if (!topo_add(li, r, true)) return false;  // topology.AddRequirements
        std::vector<int64_t> requests(R);
        for (int k = 0; k < R; k++) requests[k] = nc.requests[k] + pod.req[k];
        std::vector<int> remaining = filter(nc.options, r, requests, &r);
        if (remaining.empty()) return false;
        std::vector<int> held;
        if (resv_on && !offerings_to_reserve(nc, remaining, r, held)) return false;
        nc.pods.push_back(li);
        nc.options.swap(remaining);
        nc.requests.swap(requests);
        nc.reqs = std::move(r);
        if (resv_on) commit_reservations(nc, held);
        topo_record(li, nc.reqs, tm.taints, true);
        return true;
    }

    // NodeClaim.Add's reservation step: every available reserved offering of the remaining instance types that the
    // updated requirements are compatible with is reserved for this NodeClaim's hostname (Reserve is idempotent for an
    // ID the host already holds; otherwise it takes one unit of the ID's capacity, if any is left).  Strict mode fails
    // the Add when a compatible reserved offering exists but none can be reserved, or when the NodeClaim held
    // reservations and the updated constraints leave none (ReservedOfferingError).  Read-only: the IDs the Add would
    // hold are returned, commit_reservations applies them.
    bool offerings_to_reserve(const NodeClaim& nc, const std::vector<int>& remaining, const Reqs& r,
                              std::vector<int>& held) const {
        bool has = false;
        for (int t : remaining)
            for (auto& o : ty(t).offerings) {
                if (o.rid < 0 || !o.available) continue;
                if (!reqs_compatible(D, r, o.reqs, true)) continue;
                has = true;
                if (std::binary_search(nc.held.begin(), nc.held.end(), o.rid) || rcap[o.rid] > 0) held.push_back(o.rid);
            }
        std::sort(held.begin(), held.end());
        held.erase(std::unique(held.begin(), held.end()), held.end());
        if (resv_strict) {
            if (has && held.empty()) return false;
            if (!nc.held.empty() && held.empty()) return false;
        }
        return true;
    }
    // Reserve the newly held IDs, Release the IDs no longer compatible.
    void commit_reservations(NodeClaim& nc, std::vector<int>& held) {
        for (int id : held)
            if (!std::binary_search(nc.held.begin(), nc.held.end(), id)) rcap[id]--;
        for (int id : nc.held)
            if (!std::binary_search(held.begin(), held.end(), id)) rcap[id]++;
        nc.held.swap(held);
    }

    // ExistingNode.Add: Taints.ToleratesPod, Fits(requests + pod, available), Compatible (no undefined-label
    // allowance), then requirements.Add and topology.  On success `out` is the updated node (the caller records it).
    bool existing_try(const ExistingNode& n, int li, ExistingNode& out) {
        const Pod& pod = pod_at(li);
        const PodClass& pc = cls_of(li);
        if (!tolerates_all(n.taints, pc.tols)) return false;
        std::vector<int64_t> requests(R);
        for (int k = 0; k < R; k++) requests[k] = n.requests[k] + pod.req[k];
        if (!fits(requests, n.available)) return false;
        Reqs r = n.reqs;
        if (!reqs_compatible(D, r, pc.reqs, false)) return false;
        r.add_all(D, pc.reqs);
        if (!topo_add(li, r, false)) return false;
        out.taints = n.taints;
        out.available = n.available;
        out.host = n.host;
        out.requests.swap(requests);
        out.reqs = std::move(r);
        return true;
    }

    // sort.Slice(s.newNodeClaims, func(a, b int) bool { return len(a.Pods) < len(b.Pods) })
    struct SliceAdaptor {
        Solver* s;
        int size() const { return (int)s->newNodeClaims.size(); }
        bool less(int i, int j) const {
            return s->ncs[s->newNodeClaims[i]].pods.size() < s->ncs[s->newNodeClaims[j]].pods.size();
        }
        void swap(int i, int j) { std::swap(s->newNodeClaims[i], s->newNodeClaims[j]); }
    };

    bool add(int li) {
        for (int j : ex_idx) {
            stats.existing_evals++;
            auto it = ex_mod.find(j);
            const ExistingNode& n = it != ex_mod.end() ? it->second : (*ex_base)[j];
            ExistingNode upd;
            if (existing_try(n, li, upd)) {
                topo_record(li, upd.reqs, upd.taints, false);
                ex_mod[j] = std::move(upd);
                pod_result[li] = KP_POD_EXISTING(j);
                return true;
            }
        }
        SliceAdaptor sa{this};
        go_sort_slice(sa);
        stats.nodeclaim_candidates_scanned += (int64_t)newNodeClaims.size();
        const bool tr = (trace_pod >= 0 && plist[li] == trace_pod) ||
                        (trace_cls >= 0 && cls_id(li) == trace_cls);  // ORC_TRACE_POD / ORC_TRACE_CLASS diagnostics
        for (int idx : newNodeClaims) {
            stats.nodeclaim_evals++;
            if (tr) {
                std::string h;
                for (int id : ncs[idx].held) h += rid_names[id] + "(" + std::to_string(rcap[id]) + ") ";
                fprintf(stderr, "[orc trace] pod %d nc %d pods %zu opts %zu held %s\n", plist[li], idx,
                        ncs[idx].pods.size(), ncs[idx].options.size(), h.c_str());
            }
            if (nodeclaim_add(ncs[idx], li)) {
                if (tr) fprintf(stderr, "[orc trace]   -> accepted by nc %d\n", idx);
                pod_result[li] = idx;
                return true;
            }
        }
        for (size_t ti = 0; ti < tmpls.size(); ti++) {
            Template& tm = tmpls[ti];
            // filterByRemainingResources(its, remaining)
            std::vector<int> its;
            for (int t : tm.options) {
                bool viable = true;
                for (int k = 0; k < R; k++)
                    if (tm.limit_set[k] && ty(t).cap[k] > tm.remaining[k]) viable = false;
                if (viable) its.push_back(t);
            }
            if (its.empty()) continue;
            // NewNodeClaim
            NodeClaim nc;
            nc.id = (int)ncs.size();
            nc.tmpl = (int)ti;
            nc.reqs = tm.reqs;
            nc.host = -2 - next_host++;  // hostname-placeholder-%04d (registered in every hostname group)
            Req hr = host_req;
            hr.values = {nc.host};
            nc.reqs.add(D, hr);
            nc.options = its;
            nc.requests = tm.daemon;
            stats.template_evals++;
            if (!nodeclaim_add(nc, li)) continue;
            // subtractMax(remaining, nodeClaim.InstanceTypeOptions)
            for (int k = 0; k < R; k++) {
                if (!tm.limit_set[k]) continue;
                int64_t mx = 0;
                bool first = true;
                for (int t : nc.options) {
                    if (first || ty(t).cap[k] > mx) mx = ty(t).cap[k];
                    first = false;
                }
                tm.remaining[k] -= mx;
            }
            ncs.push_back(std::move(nc));
            newNodeClaims.push_back((int)ncs.size() - 1);
            pod_result[li] = (int)ncs.size() - 1;
            return true;
        }
        return false;
    }

    // Topology.Update keeps topologyGroups[hash]: the first owner's TopologyGroup, later owners only AddOwner().  Every
    // (class, term) group of the identity takes the first owner's selector, minDomains, node filter and tolerations and
    // its domains as buildDomainGroups left them for that owner (countDomains follows).
    void adopt(int ident, int cls) {
        int src = -1;
        for (int gi : ident_groups[ident])
            if (groups_dg[gi].owner == cls) {
                src = gi;
                break;
            }
        if (src < 0) return;
        const TopoGroup& f = groups_dg[src];
        for (int gi : ident_groups[ident]) {
            TopoGroup& g = groups[gi];
            g.sem = cls;
            g.min_domains = f.min_domains;
            g.sel = f.sel;
            g.cnt = f.cnt;
        }
    }
    // per class: the groups that constrain its pods (owned forward groups, inverse groups that select it) and those that
    // count them (forward groups that select it, owned inverse groups)
    void index_groups() {
        const int C = (int)cp->size();
        t_cons.assign(C, {});
        t_rec.assign(C, {});
        for (int gi = 0; gi < (int)groups.size(); gi++) {
            const TopoGroup& g = groups[gi];
            for (int c = 0; c < C; c++) {
                if (g.inverse) {
                    if (g.sel[c]) t_cons[c].push_back(gi);  // getMatchingTopologies: inverse groups that select the pod
                    if (g.owner == c) t_rec[c].push_back(gi);
                } else {
                    if (g.owner == c) t_cons[c].push_back(gi);
                    if (g.sel[c]) t_rec[c].push_back(gi);
                }
            }
        }
    }
    // countDomains / updateInverseAffinities for one pod of class b bound to existing node j (every group, or only
    // those of identity `only`)
    void count_bound(int j, int b, int only) {
        const ExistingNode& n = (*ex_base)[j];
        for (TopoGroup& g : groups) {
            if (only >= 0 && g.ident != only) continue;
            if (g.inverse ? g.owner != b : !g.sel[b]) continue;
            if (!g.inverse && g.type == KP_TOPO_SPREAD) {
                const PodClass& fc = (*cp)[g.sem];
                if (g.aff_pol == KP_POLICY_HONOR && !filter_matches(fc, n.reqs, false)) continue;
                if (g.taint_pol == KP_POLICY_HONOR && !tolerates_all(n.taints, fc.tols)) continue;
            }
            int dom;
            if (g.host) {
                dom = n.host;
            } else {
                auto it = n.reqs.m.find(g.key);
                if (it == n.reqs.m.end() || it->second.complement || it->second.values.size() != 1) continue;  // unlabeled
                dom = it->second.values[0];
            }
            g.cnt[dom]++;
        }
    }
    // NewTopology over this simulation's pods (plist, input order): each identity is created from the first pod whose
    // spec owns it, then countDomains over bound_pods.  An identity no pod owns yet keeps its per-class groups until a
    // relaxation creates it (birth).
    void new_topology() {
        groups = groups_dg;
        if (groups.empty()) return;
        std::vector<int> firstpos(cp->size(), INT32_MAX);
        for (int li = (int)plist.size() - 1; li >= 0; li--) firstpos[pod_at(li).cls] = li;
        for (int I = 0; I < (int)ident_groups.size(); I++) {
            int best = -1;
            for (int gi : ident_groups[I]) {
                const int o = groups_dg[gi].owner;
                if (o < n_input && firstpos[o] != INT32_MAX && (best < 0 || firstpos[o] < firstpos[best])) best = o;
            }
            if (best >= 0) adopt(I, best);
        }
        index_groups();
        for (auto& bp : bound_pods) count_bound(bp.first, bp.second, -1);
    }
    // Topology.Update of a pod relaxed into class cls creates the late identities it owns that no pod created yet: from
    // this pod's spec, countDomains over the bound pods only (the pods of this Solve are excluded)
    void birth(int cls) {
        const uint64_t fresh = cls_birth[cls] & ~born;
        if (!fresh) return;
        born |= fresh;
        for (uint64_t x = fresh; x; x &= x - 1) {
            const int I = late_ident[__builtin_ctzll(x)];
            adopt(I, cls);
            for (auto& bp : bound_pods) count_bound(bp.first, bp.second, I);
        }
        index_groups();
    }

    void solve() {
        // NewTopology creates the groups the batch's pods own; Topology.Update those of a relaxed pod's new spec
        born = ~0ull;
        if (n_late > 0 && !getenv("ORC_NO_LATE")) {  // ORC_NO_LATE (diagnostics): every group counts from the start
            born = 0;
            for (int li = 0; li < (int)plist.size(); li++) born |= cls_birth[pod_at(li).cls];
        }
        // NewQueue: sort.Slice(pods, byCPUAndMemoryDescending) — a total order (Kubernetes UIDs are unique).  Inputs
        // without UIDs (kp_pods_view.uids NULL) keep their input order on ties, as the device's stable radix passes do.
        const int n = (int)plist.size();
        std::vector<int> order(n);
        for (int i = 0; i < n; i++) order[i] = i;
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
            const Pod& l = pod_at(a);
            const Pod& r = pod_at(b);
            if (l.req[cpu_axis] != r.req[cpu_axis]) return l.req[cpu_axis] > r.req[cpu_axis];
            if (l.req[mem_axis] != r.req[mem_axis]) return l.req[mem_axis] > r.req[mem_axis];
            if (l.ts != r.ts) return l.ts < r.ts;
            return l.uid < r.uid;
        });
        std::deque<int> q(order.begin(), order.end());
        std::unordered_map<int, int> lastLen;
        pcls.resize(n);
        for (int i = 0; i < n; i++) pcls[i] = pod_at(i).cls;
        pod_result.assign(n, KP_POD_UNSCHEDULABLE);
        pod_order.assign(n, -1);
        for (;;) {
            if (q.empty()) break;
            int li = q.front();
            auto it = lastLen.find(li);
            if (it != lastLen.end() && it->second == (int)q.size()) break;
            q.pop_front();
            stats.pods_popped++;
            if (add(li)) {
                pod_order[li] = placements++;
                continue;
            }
            // preferences.Relax, then Queue.Push(pod, relaxed): a relaxed pod clears lastLen (and Topology.Update /
            // updateCachedPodData take its new spec: the next relaxation stage of its class)
            const int nx = relax_next.empty() ? -1 : relax_next[cls_id(li)];
            q.push_back(li);
            if (nx >= 0) {
                pcls[li] = nx;
                if (n_late > 0) birth(nx);
                lastLen.clear();
            } else {
                lastLen[li] = (int)q.size();
            }
        }
    }

    // Cheapest available offering compatible with reqs (OrderByPrice key); MaxFloat64 when none.
    double cheapest(int t, const Reqs& reqs) const {
        double price = DBL_MAX;
        bool any = false;
        for (auto& o : ty(t).offerings) {
            if (!o.available || !reqs_compatible(D, reqs, o.reqs, true)) continue;
            if (!any || o.price < price) price = o.price;
            any = true;
        }
        return any ? price : DBL_MAX;
    }

    // Solve's FinalizeScheduling + Results.TruncateInstanceTypes(maxInstanceTypes): hostname removed,
    // InstanceTypes.Truncate = OrderByPrice(reqs) then the first max types, SatisfiesMinValues on the kept list
    // (a NodeClaim that fails it is dropped and its pods get errors).
    void finalize(int max_types) {
        for (auto& nc : ncs) {
            nc.reqs.m.erase(hostname_key);
            // FinalizeScheduling: a NodeClaim holding reservations gets ReservationIDLabel In [held IDs]
            if (!nc.held.empty()) {
                std::vector<std::string> ids;
                for (int id : nc.held) ids.push_back(rid_names[id]);
                nc.reqs.add(D, new_req(D, resv_key, OP_IN, ids, false, 0));
            }
            std::vector<std::pair<double, int>> keyed;
            for (int t : nc.options) keyed.push_back({cheapest(t, nc.reqs), t});
            std::sort(keyed.begin(), keyed.end(), [&](const std::pair<double, int>& a, const std::pair<double, int>& b) {
                if (a.first == b.first) return ty(a.second).name < ty(b.second).name;
                return a.first < b.first;
            });
            std::vector<int> tr;
            for (auto& kv : keyed) tr.push_back(kv.second);
            if (max_types > 0 && (int)tr.size() > max_types) tr.resize(max_types);
            if (nc.reqs.has_min_values() && !satisfies_min_values(tr, nc.reqs)) {
                nc.valid = false;
                for (int li : nc.pods) {
                    pod_result[li] = KP_POD_UNSCHEDULABLE;
                    pod_order[li] = -1;
                }
            }
            nc.truncated = tr;
        }
    }
    int cpu_axis = 0, mem_axis = 1;
};

static std::vector<std::string> strs(const char* const* v, int n) {
    std::vector<std::string> o;
    for (int i = 0; i < n; i++) o.emplace_back(v[i] ? v[i] : "");
    return o;
}

static bool build_reqs(Dict& D, const kp_requirement* rs, int n, Reqs& out) {
    for (int i = 0; i < n; i++) {
        const kp_requirement& r = rs[i];
        if (!r.key || r.op < 0 || r.op > 5) return false;
        int k = D.key(normalize_label(r.key));
        out.add(D, new_req(D, k, (Op)r.op, strs(r.values, r.n_values), r.min_values >= 0, r.min_values));
    }
    return true;
}

}  // namespace orc

using namespace orc;

struct orc_result {
    std::vector<NodeClaim> ncs;
    Dict D;
};

// Input views → NewScheduler state (catalog rows, classes, pods, NodeClaimTemplates in weight order, existing nodes),
// then NewTopology (domain groups, topology groups, counts of the bound pods).
static kp_status build_topology(Solver& s, const kp_solve_input* in, const std::vector<PoolDomains>& pools);

static kp_status parse_into(Solver& s, const kp_catalog_view* cat, const kp_solve_input* in, int pref_policy) {
    Dict& D = s.D;
    const int T = cat->n_types, R = cat->n_resources;
    s.R = R;
    s.cpu_axis = s.mem_axis = -1;
    for (int r = 0; r < R; r++) {
        if (!strcmp(cat->resource_names[r], "cpu")) s.cpu_axis = r;
        if (!strcmp(cat->resource_names[r], "memory")) s.mem_axis = r;
    }
    if (s.cpu_axis < 0 || s.mem_axis < 0) return KP_E_INVALID;
    s.hostname_key = D.key("kubernetes.io/hostname");
    s.host_req = new_req(D, s.hostname_key, OP_IN, {"hostname-placeholder"}, false, 0);
    s.resv_key = D.key("karpenter.k8s.aws/capacity-reservation-id");
    // catalog → []*cloudprovider.InstanceType
    s.own_types.resize(T);
    for (int t = 0; t < T; t++) {
        InstanceType& it = s.own_types[t];
        it.name = cat->type_names[t];
        it.cap.assign(cat->capacity + (size_t)t * R, cat->capacity + (size_t)(t + 1) * R);
        it.alloc.assign(cat->allocatable + (size_t)t * R, cat->allocatable + (size_t)(t + 1) * R);
        for (int k = 0; k < cat->n_label_keys; k++) {
            int st = cat->label_state[(size_t)t * cat->n_label_keys + k];
            if (st == KP_LABEL_ABSENT) continue;
            int key = D.key(normalize_label(cat->label_keys[k]));
            if (st == KP_LABEL_DOES_NOT_EXIST) {
                it.reqs.add(D, new_req(D, key, OP_DNE, {}, false, 0));
            } else {
                int o0 = cat->label_offsets[(size_t)t * cat->n_label_keys + k];
                int o1 = cat->label_offsets[(size_t)t * cat->n_label_keys + k + 1];
                it.reqs.add(D, new_req(D, key, OP_IN, strs(cat->label_values + o0, o1 - o0), false, 0));
            }
        }
    }
    for (int o = 0; o < cat->n_offerings; o++) {
        int t = cat->offering_type[o];
        if (t < 0 || t >= T) return KP_E_INVALID;
        Offering of;
        of.price = cat->offering_price[o];
        of.available = cat->offering_available[o] != 0;
        for (int k = 0; k < cat->n_offering_keys; k++) {
            int st = cat->offering_label_state[(size_t)o * cat->n_offering_keys + k];
            if (st == KP_LABEL_ABSENT) continue;
            int key = D.key(normalize_label(cat->offering_keys[k]));
            if (st == KP_LABEL_DOES_NOT_EXIST)
                of.reqs.add(D, new_req(D, key, OP_DNE, {}, false, 0));
            else
                of.reqs.add(D, new_req(D, key, OP_IN, {cat->offering_label_values[(size_t)o * cat->n_offering_keys + k]}, false, 0));
        }
        // reserved offerings (offering.go:164-194) carry ReservationIDLabel In [id]; NewReservationManager keeps the
        // least ReservationCapacity per ID
        auto rit = of.reqs.m.find(s.resv_key);
        if (rit != of.reqs.m.end() && !rit->second.complement && rit->second.values.size() == 1) {
            const std::string id = D.vals[s.resv_key][rit->second.values[0]];
            const int rc = cat->offering_reservation_capacity ? cat->offering_reservation_capacity[o] : 0;
            int ix = -1;
            for (size_t i = 0; i < s.rid_names.size(); i++)
                if (s.rid_names[i] == id) ix = (int)i;
            if (ix < 0) {
                ix = (int)s.rid_names.size();
                s.rid_names.push_back(id);
                s.rcap.push_back(rc);
            } else {
                s.rcap[ix] = std::min(s.rcap[ix], rc);
            }
            of.rid = ix;
        }
        s.own_types[t].offerings.push_back(std::move(of));
    }
    s.resv_on = s.resv_on && !s.rid_names.empty();
    // pod classes, expanded into preferences.Relax stages: stage 0 of class c is own_classes[c]; further stages are
    // appended, relax_next links them (kp_pod_class comment in kpsim.h; preferences.go, recalled)
    bool tol_pns = false;  // NewScheduler: some NodePool template carries a PreferNoSchedule taint
    for (int i = 0; i < in->n_nodepools; i++)
        for (int j = 0; j < in->nodepools[i].n_taints; j++)
            if (in->nodepools[i].taints[j].effect && !strcmp(in->nodepools[i].taints[j].effect, "PreferNoSchedule"))
                tol_pns = true;
    auto parse_term = [&](const kp_topology_term& x, const std::string& ns, TopoTerm& t) -> kp_status {
        if (x.type < KP_TOPO_SPREAD || x.type > KP_TOPO_ANTI_AFFINITY || !x.topology_key) return KP_E_INVALID;
        t.type = x.type;
        t.key = D.key(normalize_label(x.topology_key));
        t.max_skew = x.type == KP_TOPO_SPREAD ? x.max_skew : INT32_MAX;
        if (x.type == KP_TOPO_SPREAD && x.max_skew <= 0) return KP_E_INVALID;
        t.min_domains = x.type == KP_TOPO_SPREAD && x.min_domains > 0 ? x.min_domains : -1;
        t.aff_pol = x.type == KP_TOPO_SPREAD ? x.node_affinity_policy : KP_POLICY_IGNORE;
        t.taint_pol = x.type == KP_TOPO_SPREAD ? x.node_taints_policy : KP_POLICY_IGNORE;
        t.preferred = x.type == KP_TOPO_SPREAD ? x.when_unsatisfiable == KP_SCHEDULE_ANYWAY : x.weight > 0;
        t.sel.nil = x.n_selector < 0;
        for (int j = 0; j < x.n_selector; j++) {
            const kp_requirement& q = x.selector[j];
            if (!q.key || q.op < KP_OP_IN || q.op > KP_OP_DOES_NOT_EXIST) return KP_E_INVALID;
            LabelSel::Term st;
            st.key = q.key;
            st.op = q.op;
            st.values = strs(q.values, q.n_values);
            t.sel.terms.push_back(st);
        }
        if (x.type == KP_TOPO_SPREAD || x.n_namespaces <= 0) t.namespaces = {ns};
        else t.namespaces = strs(x.namespaces, x.n_namespaces);
        return KP_OK;
    };
    // The spec state a pod's Relax steps walk through.
    struct Spec {
        int req_first = 0;           // first remaining required node-affinity term
        std::vector<int> pnode;      // remaining preferred node-affinity terms, heaviest first (stable)
        std::vector<int> paff, panti;  // remaining preferred pod (anti-)affinity terms, heaviest first (SliceStable)
        std::vector<int> spreads;    // TopologySpreadConstraints in spec order (swap-with-last removal)
        bool pns = false;            // the PreferNoSchedule toleration was added
    };
    const int C0 = in->n_classes;
    s.own_classes.clear();
    s.own_classes.resize(C0);
    s.relax_next.assign(C0, -1);
    bool any_relax = false;
    std::vector<std::pair<int, Spec>> work;  // (class id, spec) whose Relax step is still to be derived
    for (int c = 0; c < C0; c++) {
        const kp_pod_class& pc = in->classes[c];
        Spec sp;
        // newPodRequirements: sort.Slice(preferred, weight desc) in place — Go's pdqsort (insertion sort up to 12
        // terms); the sorted slice stays as it is under later sorts and Relax's SliceStable
        for (int i = 0; i < pc.n_preferred_terms; i++) sp.pnode.push_back(i);
        {
            struct D {
                std::vector<int>& v;
                const kp_pod_class& pc;
                int size() const { return (int)v.size(); }
                bool less(int a, int b) const { return pc.preferred_terms[v[a]].weight > pc.preferred_terms[v[b]].weight; }
                void swap(int a, int b) { std::swap(v[a], v[b]); }
            } d{sp.pnode, pc};
            orc::go_sort_slice(d);
        }
        for (int i = 0; i < pc.n_topology; i++) {
            const kp_topology_term& x = pc.topology[i];
            if (x.type == KP_TOPO_SPREAD) sp.spreads.push_back(i);
            else if (x.weight > 0) (x.type == KP_TOPO_AFFINITY ? sp.paff : sp.panti).push_back(i);
        }
        for (auto* v : {&sp.paff, &sp.panti})
            std::stable_sort(v->begin(), v->end(), [&](int a, int b) { return pc.topology[a].weight > pc.topology[b].weight; });
        work.push_back({c, sp});
    }
    auto has_pns_tol = [](const kp_pod_class& pc) {  // Toleration.MatchToleration of {Exists, PreferNoSchedule}
        for (int i = 0; i < pc.n_tolerations; i++) {
            const kp_toleration& t = pc.tolerations[i];
            if (t.op == KP_TOL_EXISTS && (!t.key || !*t.key) && (!t.value || !*t.value) && t.effect &&
                !strcmp(t.effect, "PreferNoSchedule"))
                return true;
        }
        return false;
    };
    std::vector<int> origin(C0);  // class id -> input class
    for (int c = 0; c < C0; c++) origin[c] = c;
    for (size_t w = 0; w < work.size(); w++) {
        const int id = work[w].first;
        const Spec sp = work[w].second;
        const int oc = origin[id];
        const kp_pod_class& pc = in->classes[oc];
        // the effective PodClass of this spec
        PodClass& out = s.own_classes[id];
        if (!build_reqs(D, pc.requirements, pc.n_requirements, out.reqs)) return KP_E_INVALID;
        if (pc.n_required_terms > 0 &&
            !build_reqs(D, pc.required_terms[sp.req_first].requirements, pc.required_terms[sp.req_first].n_requirements, out.reqs))
            return KP_E_INVALID;
        if (pc.n_required_terms == 0) {
            out.filter.emplace_back();
            if (!build_reqs(D, pc.requirements, pc.n_requirements, out.filter.back())) return KP_E_INVALID;
        }
        for (int i = sp.req_first; i < pc.n_required_terms; i++) {
            out.filter.emplace_back();
            if (!build_reqs(D, pc.requirements, pc.n_requirements, out.filter.back()) ||
                !build_reqs(D, pc.required_terms[i].requirements, pc.required_terms[i].n_requirements, out.filter.back()))
                return KP_E_INVALID;
        }
        if (pref_policy == KP_PREFERENCE_RESPECT && !sp.pnode.empty()) {
            out.strict = out.reqs;
            out.has_strict = true;
            if (!build_reqs(D, pc.preferred_terms[sp.pnode[0]].requirements, pc.preferred_terms[sp.pnode[0]].n_requirements, out.reqs))
                return KP_E_INVALID;
        }
        for (int i = 0; i < pc.n_tolerations; i++) {
            Toleration t;
            t.key = pc.tolerations[i].key ? pc.tolerations[i].key : "";
            t.op = pc.tolerations[i].op;
            t.value = pc.tolerations[i].value ? pc.tolerations[i].value : "";
            t.effect = pc.tolerations[i].effect ? pc.tolerations[i].effect : "";
            out.tols.push_back(t);
        }
        if (sp.pns) {
            Toleration t;
            t.op = KP_TOL_EXISTS;
            t.effect = "PreferNoSchedule";
            out.tols.push_back(t);
        }
        if (pc.namespace_name) out.ns = pc.namespace_name;
        for (int l = 0; l < pc.n_labels; l++)
            out.labels[pc.label_keys[l] ? pc.label_keys[l] : ""] = pc.label_values[l] ? pc.label_values[l] : "";
        auto add_term = [&](int i) -> kp_status {
            const kp_topology_term& x = pc.topology[i];
            const bool preferred = x.type == KP_TOPO_SPREAD ? x.when_unsatisfiable == KP_SCHEDULE_ANYWAY : x.weight > 0;
            if (preferred && pref_policy == KP_PREFERENCE_IGNORE) return KP_OK;  // Ignore drops preferences
            TopoTerm t;
            kp_status st = parse_term(x, out.ns, t);
            if (st == KP_OK) out.terms.push_back(t);
            return st;
        };
        for (int i : sp.spreads)
            if (kp_status st = add_term(i)) return st;
        for (int i = 0; i < pc.n_topology; i++)
            if (pc.topology[i].type != KP_TOPO_SPREAD && pc.topology[i].weight <= 0)
                if (kp_status st = add_term(i)) return st;
        for (auto* v : {&sp.paff, &sp.panti})
            for (int i : *v)
                if (kp_status st = add_term(i)) return st;
        // Preferences.Relax: the first relaxation that applies
        Spec nx = sp;
        bool relaxed = true;
        if (pc.n_required_terms - sp.req_first > 1) {
            nx.req_first++;                                  // removeRequiredNodeAffinityTerm
        } else if (!sp.paff.empty()) {
            nx.paff.erase(nx.paff.begin());                  // removePreferredPodAffinityTerm
        } else if (!sp.panti.empty()) {
            nx.panti.erase(nx.panti.begin());                // removePreferredPodAntiAffinityTerm
        } else if (!sp.pnode.empty()) {
            nx.pnode.erase(nx.pnode.begin());                // removePreferredNodeAffinityTerm
        } else {
            relaxed = false;
            for (size_t i = 0; i < sp.spreads.size() && !relaxed; i++)
                if (pc.topology[sp.spreads[i]].when_unsatisfiable == KP_SCHEDULE_ANYWAY) {  // removeTopologySpreadScheduleAnyway
                    nx.spreads[i] = nx.spreads.back();
                    nx.spreads.pop_back();
                    relaxed = true;
                }
            if (!relaxed && tol_pns && !sp.pns && !has_pns_tol(pc)) {  // toleratePreferNoScheduleTaints
                nx.pns = true;
                relaxed = true;
            }
        }
        if (relaxed) {
            const int nid = (int)s.own_classes.size();
            s.own_classes.emplace_back();
            s.relax_next.push_back(-1);
            origin.push_back(oc);
            s.relax_next[id] = nid;
            work.push_back({nid, nx});
            any_relax = true;
        }
    }
    if (!any_relax) s.relax_next.clear();
    s.cls_origin = origin;
    s.n_input = C0;
    // pods
    const kp_pods_view& pv = in->pods;
    s.own_pods.resize(pv.n_pods);
    for (int p = 0; p < pv.n_pods; p++) {
        Pod& pod = s.own_pods[p];
        pod.cls = pv.class_id[p];
        if (pod.cls < 0 || pod.cls >= in->n_classes) return KP_E_INVALID;
        pod.req.assign(pv.requests + (size_t)p * R, pv.requests + (size_t)(p + 1) * R);
        pod.ts = pv.creation_ns ? pv.creation_ns[p] : 0;
        pod.uid = pv.uids && pv.uids[p] ? pv.uids[p] : "";
    }
    // NodePools → NodeClaimTemplates, OrderByWeight (weight desc, name asc)
    std::vector<int> npo(in->n_nodepools);
    for (int i = 0; i < in->n_nodepools; i++) npo[i] = i;
    std::sort(npo.begin(), npo.end(), [&](int a, int b) {
        const kp_nodepool& x = in->nodepools[a];
        const kp_nodepool& y = in->nodepools[b];
        if (x.weight != y.weight) return x.weight > y.weight;
        return strcmp(x.name, y.name) < 0;
    });
    std::vector<PoolDomains> pools(in->n_nodepools);
    for (int i : npo) {
        const kp_nodepool& np = in->nodepools[i];
        Template tm;
        tm.np_index = i;
        tm.name = np.name;
        tm.weight = np.weight;
        if (!build_reqs(D, np.requirements, np.n_requirements, tm.reqs)) return KP_E_INVALID;
        for (int j = 0; j < np.n_taints; j++)
            tm.taints.push_back({np.taints[j].key ? np.taints[j].key : "", np.taints[j].value ? np.taints[j].value : "",
                                 np.taints[j].effect ? np.taints[j].effect : ""});
        pools[i].reqs = tm.reqs;
        pools[i].taints = tm.taints;
        tm.daemon.assign(R, 0);
        if (np.daemon_overhead) tm.daemon.assign(np.daemon_overhead, np.daemon_overhead + R);
        tm.limit_set.assign(R, 0);
        tm.remaining.assign(R, 0);
        if (np.limit_set) {
            tm.limit_set.assign(np.limit_set, np.limit_set + R);
            tm.remaining.assign(np.limit_remaining, np.limit_remaining + R);
        }
        std::vector<int> rows;
        if (np.n_types < 0) {
            for (int t = 0; t < T; t++) rows.push_back(t);
        } else {
            for (int j = 0; j < np.n_types; j++) rows.push_back(np.type_index[j]);
        }
        pools[i].rows = rows;
        // NewScheduler: nct.InstanceTypeOptions = filterInstanceTypesByRequirements(its, nct.Requirements, {}, {}, {})
        std::vector<int64_t> zero(R, 0);
        // Fits({}, alloc) only rejects negative allocatable; emulate with an all-zero request
        tm.options = s.filter(rows, tm.reqs, zero);
        if (tm.options.empty()) continue;  // "skipping, nodepool requirements filtered out all instance types"
        s.tmpls.push_back(std::move(tm));
    }
    // existing nodes
    for (int j = 0; j < in->n_existing; j++) {
        const kp_existing_node& en = in->existing[j];
        ExistingNode n;
        for (int l = 0; l < en.n_labels; l++) {
            int k = D.key(normalize_label(en.label_keys[l]));
            n.reqs.add(D, new_req(D, k, OP_IN, {en.label_values[l]}, false, 0));
        }
        n.reqs.add(D, new_req(D, s.hostname_key, OP_IN, {en.name ? en.name : ""}, false, 0));
        n.host = D.value(s.hostname_key, en.name ? en.name : "");
        for (int l = 0; l < en.n_taints; l++)
            n.taints.push_back({en.taints[l].key ? en.taints[l].key : "", en.taints[l].value ? en.taints[l].value : "",
                                en.taints[l].effect ? en.taints[l].effect : ""});
        n.available.assign(en.available, en.available + R);
        n.requests.assign(R, 0);
        if (en.requests) n.requests.assign(en.requests, en.requests + R);
        s.own_existing.push_back(std::move(n));
    }
    return build_topology(s, in, pools);
}

// NewTopology: buildDomainGroups over every NodePool × its instance types, one forward group per topology term of a
// class (newForTopologies / newForAffinities) and one inverse group per required anti-affinity term
// (updateInverseAntiAffinity), then countDomains over the bound pods and the bound pods' inverse anti-affinities.
static kp_status build_topology(Solver& s, const kp_solve_input* in, const std::vector<PoolDomains>& pools) {
    Dict& D = s.D;
    const int C = (int)s.own_classes.size();
    bool any = false;
    for (auto& pc : s.own_classes) any = any || !pc.terms.empty();
    if (!any) return KP_OK;
    // buildDomainGroups: key → domain → taint sets of the NodePools that offer it
    std::map<int, std::map<int, std::vector<int>>> dg;  // key → domain → pools
    auto domains_of = [&](int key) -> const std::map<int, std::vector<int>>& {
        auto it = dg.find(key);
        if (it != dg.end()) return it->second;
        std::map<int, std::vector<int>>& m = dg[key];
        for (int p = 0; p < (int)pools.size(); p++) {
            const PoolDomains& pd = pools[p];
            for (int t : pd.rows) {
                // requirements = NodePool requirements (+ template labels), Add(it.Requirements)
                const InstanceType& it = s.ty(t);
                const bool hp = pd.reqs.has(key), ht = it.reqs.has(key);
                if (!hp && !ht) continue;
                Req x = hp && ht ? req_intersection(D, it.reqs.m.at(key), pd.reqs.m.at(key)) : (hp ? pd.reqs.m.at(key) : it.reqs.m.at(key));
                for (int v : x.values) m[v].push_back(p);  // requirement.Values()
            }
            if (pd.reqs.has(key) && pd.reqs.m.at(key).Operator() == OP_IN)
                for (int v : pd.reqs.m.at(key).values) m[v].push_back(p);
        }
        return m;
    };
    auto tolerated_domain = [&](const std::vector<int>& ps, int cls) {  // ForEachDomain with NodeTaintsPolicy Honor
        for (int p : ps)
            if (tolerates_all(pools[p].taints, s.own_classes[cls].tols)) return true;
        return false;
    };
    for (int c = 0; c < C; c++) {
        const PodClass& pc = s.own_classes[c];
        for (const TopoTerm& t : pc.terms) {
            for (int inv = 0; inv < 2; inv++) {
                // updateInverseAntiAffinity: only required anti-affinity terms get an inverse group
                if (inv && (t.type != KP_TOPO_ANTI_AFFINITY || t.preferred)) break;
                TopoGroup g;
                g.type = t.type;
                g.key = t.key;
                g.host = t.key == s.hostname_key;
                g.inverse = inv == 1;
                g.owner = c;
                g.sem = c;
                g.max_skew = t.max_skew;
                g.min_domains = t.min_domains;
                g.aff_pol = t.aff_pol;
                g.taint_pol = t.taint_pol;
                g.sel.assign(C, 0);
                for (int o = 0; o < C; o++) {
                    const PodClass& q = s.own_classes[o];
                    g.sel[o] = std::find(t.namespaces.begin(), t.namespaces.end(), q.ns) != t.namespaces.end() &&
                               t.sel.matches(q.labels);
                }
                if (!g.host)
                    for (auto& kv : domains_of(t.key))
                        if (t.type != KP_TOPO_SPREAD || t.taint_pol != KP_POLICY_HONOR || tolerated_domain(kv.second, c))
                            g.cnt[kv.first] = 0;
                s.groups.push_back(std::move(g));
            }
        }
    }
    // Topology.Update creates a group (countDomains counts the bound pods) unless one of equal TopologyGroup.Hash()
    // exists: key, type, namespaces, selector, maxSkew and the node filter — the requirement KEY sets of the
    // nodeSelector with each remaining required term (hashstructure skips unexported fields: no values), the
    // policies and the tolerations; slices hash as the XOR of their elements (SlicesAsSets), so pairs cancel.  An
    // identity that a relaxed spec owns while its input class's stage 0 does not can only be created by a relaxation:
    // it is "late" and records nothing until then.
    {
        auto parity = [](std::vector<std::string> v) {
            std::sort(v.begin(), v.end());
            std::string o;
            for (size_t i = 0; i < v.size();) {
                size_t j = i;
                while (j < v.size() && v[j] == v[i]) j++;
                if ((j - i) & 1) o += v[i] + "\x1f";
                i = j;
            }
            return o;
        };
        std::map<std::string, int> ids;
        std::vector<int> gid(s.groups.size());
        size_t gi = 0;
        for (int c = 0; c < C; c++) {
            const PodClass& pc = s.own_classes[c];
            for (const TopoTerm& t : pc.terms) {
                std::set<std::string> nss(t.namespaces.begin(), t.namespaces.end());
                std::string base = std::to_string(t.type) + "\x1e" + std::to_string(t.key) + "\x1e";
                for (auto& n : nss) base += n + "\x1f";
                base += "\x1e";
                if (t.sel.nil) {
                    base += "nil";
                } else {
                    std::vector<std::string> el;
                    for (auto& q : t.sel.terms) el.push_back(q.key + "\x1d" + std::to_string(q.op) + "\x1d" + parity(q.values));
                    base += "sel" + parity(el);
                }
                base += "\x1e" + std::to_string(t.max_skew) + "\x1e";
                for (int inv = 0; inv < 2; inv++) {
                    if (inv && (t.type != KP_TOPO_ANTI_AFFINITY || t.preferred)) break;
                    std::string id = (inv ? "I\x1e" : "F\x1e") + base;
                    if (t.type == KP_TOPO_SPREAD) {
                        std::vector<std::string> ks, tl;
                        for (const Reqs& f : pc.filter) {
                            std::string k;
                            for (auto& kv : f.m) k += std::to_string(kv.first) + "\x1c";
                            ks.push_back(k);
                        }
                        for (auto& x : pc.tols) tl.push_back(x.key + "\x1d" + std::to_string(x.op) + "\x1d" + x.value + "\x1d" + x.effect);
                        id += parity(ks) + "\x1e" + std::to_string(t.aff_pol) + std::to_string(t.taint_pol) + "\x1e" + parity(tl);
                    }
                    auto it = ids.find(id);
                    int ix;
                    if (it != ids.end()) {
                        ix = it->second;
                    } else {
                        ix = (int)ids.size();
                        ids.emplace(id, ix);
                    }
                    gid[gi++] = ix;
                }
            }
        }
        const int NI = (int)ids.size();
        std::vector<std::set<int>> own0(NI);
        for (size_t g = 0; g < s.groups.size(); g++)
            if (s.groups[g].owner < s.n_input) own0[gid[g]].insert(s.groups[g].owner);
        std::vector<int> late(NI, -1);
        for (size_t g = 0; g < s.groups.size(); g++) {
            const int o = s.groups[g].owner;
            if (o < s.n_input || late[gid[g]] >= 0 || own0[gid[g]].count(s.cls_origin[o])) continue;
            if (s.n_late >= 64) return KP_E_UNSUPPORTED;  // shared with the device build
            late[gid[g]] = s.n_late++;
        }
        s.cls_birth.assign(C, 0);
        s.late_ident.assign(s.n_late, -1);
        s.ident_groups.assign(NI, {});
        for (size_t g = 0; g < s.groups.size(); g++) {
            s.groups[g].late = late[gid[g]];
            s.groups[g].ident = gid[g];
            s.ident_groups[gid[g]].push_back((int)g);
            if (late[gid[g]] >= 0) {
                s.cls_birth[s.groups[g].owner] |= 1ull << late[gid[g]];
                s.late_ident[late[gid[g]]] = gid[g];
            }
        }
    }
    s.groups_dg = s.groups;  // the domain groups before any pod is counted (Solver::new_topology counts)
    s.index_groups();
    // bound pods: countDomains (forward groups; node filter against the node's labels and taints) and the inverse
    // anti-affinity of bound pods (recorded at their node's domain), in Solver::new_topology once the pods are known
    const int E = (int)s.own_existing.size();
    for (int i = 0; i < in->n_bound; i++) {
        const int j = in->bound_node[i], b = in->bound_class[i];
        if (j < 0 || j >= E || b < 0 || b >= C) return KP_E_INVALID;
        s.bound_pods.push_back({j, b});
    }
    return KP_OK;
}

extern "C" kp_status orc_solve_opts(const kp_catalog_view* cat, const kp_solve_input* in, const kp_device_opts* opts,
                                    kp_solve_output* out, orc_result** res_out) {
    if (!cat || !in || !out) return KP_E_INVALID;
    if (in->min_values_policy != KP_MIN_VALUES_STRICT && in->min_values_policy != KP_MIN_VALUES_BEST_EFFORT)
        return KP_E_INVALID;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    auto res = std::make_unique<orc_result>();
    Solver s(res->D);
    s.resv_on = opts ? opts->reserved_capacity != 0 : true;  // FEATURE_GATES ReservedCapacity (default on)
    s.resv_strict = true;  // provisioning: scheduling.DisableReservedCapacityFallback
    s.best_effort = in->min_values_policy == KP_MIN_VALUES_BEST_EFFORT;
    kp_status st = parse_into(s, cat, in, opts ? opts->preference_policy : KP_PREFERENCE_RESPECT);
    if (st != KP_OK) return st;
    for (int j = 0; j < (int)s.own_existing.size(); j++) s.ex_idx.push_back(j);
    const kp_pods_view& pv = in->pods;
    s.plist.resize(pv.n_pods);
    for (int p = 0; p < pv.n_pods; p++) s.plist[p] = p;
    s.new_topology();

    const auto t1 = clk::now();
    s.solve();
    const auto t2 = clk::now();
    s.finalize(in->max_instance_types);
    const auto t3 = clk::now();
    // the oracle's phases in the device's stats fields: input parsing, the Solve loop, FinalizeScheduling + Truncate
    auto ns = [](clk::time_point a, clk::time_point b) { return (double)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count(); };
    s.stats.ns_host_prep = ns(t0, t1);
    s.stats.ns_device_solve = ns(t1, t2);
    s.stats.ns_device_finalize = ns(t2, t3);
    s.stats.ns_total = ns(t0, t3);

    // outputs
    int n_nc = (int)s.ncs.size();
    int n_ids = 0;
    for (auto& nc : s.ncs) n_ids += (int)nc.truncated.size();
    out->n_nodeclaims = n_nc;
    out->n_type_ids = n_ids;
    out->stats = s.stats;
    if (n_nc > out->cap_nodeclaims || n_ids > out->cap_type_ids) return KP_E_BUFFER;
    std::vector<int> slice_pos(n_nc, -1);
    for (size_t i = 0; i < s.newNodeClaims.size(); i++) slice_pos[s.newNodeClaims[i]] = (int)i;
    int off = 0;
    for (int i = 0; i < n_nc; i++) {
        const NodeClaim& nc = s.ncs[i];
        out->nodeclaim_nodepool[i] = nc.valid ? s.tmpls[nc.tmpl].np_index : -1;
        out->nodeclaim_n_pods[i] = (int)nc.pods.size();
        if (out->nodeclaim_slice_pos) out->nodeclaim_slice_pos[i] = slice_pos[i];
        if (out->nodeclaim_n_options) out->nodeclaim_n_options[i] = (int)nc.options.size();
        out->nodeclaim_type_offset[i] = off;
        for (int t : nc.truncated) out->type_ids[off++] = t;
    }
    out->nodeclaim_type_offset[n_nc] = off;
    for (int p = 0; p < pv.n_pods; p++) {
        out->pod_result[p] = s.pod_result[p];
        if (out->pod_order) out->pod_order[p] = s.pod_order[p];
    }
    if (res_out) {
        res->ncs = std::move(s.ncs);
        *res_out = res.release();
    }
    return KP_OK;
}

extern "C" kp_status orc_solve(const kp_catalog_view* cat, const kp_solve_input* in, kp_solve_output* out,
                               orc_result** res_out) {
    return orc_solve_opts(cat, in, nullptr, out, res_out);
}

// ------------------------------------------------------------------------------------------------
// Consolidation ([core] pkg/controllers/disruption, recalled — DESIGN.md §7)
// ------------------------------------------------------------------------------------------------
namespace orc {

struct ConsCtx {
    Solver* base;
    const kp_consolidate_input* in;
    int ct_key = -1;
    Reqs ct_reserved, ct_spot, ct_od;  // NewRequirements(capacity-type In [x])
    Req spot_req;
    int v_spot = -1, v_od = -1;        // value ids in the capacity-type dictionary
};

// Offerings.Available().WorstLaunchPrice(reqs) (cloudprovider/types.go): the first capacity type in the precedence
// reserved, spot, on-demand with a compatible offering; the most expensive such offering.
static double worst_launch_price(const ConsCtx& X, int t, const Reqs& reqs) {
    const Solver& b = *X.base;
    for (const Reqs* ct : {&X.ct_reserved, &X.ct_spot, &X.ct_od}) {
        bool any = false;
        double mx = 0;
        for (auto& o : b.ty(t).offerings) {
            if (!o.available || !reqs_compatible(b.D, reqs, o.reqs, true) || !reqs_compatible(b.D, *ct, o.reqs, true))
                continue;
            if (!any || o.price > mx) mx = o.price;
            any = true;
        }
        if (any) return mx;
    }
    return DBL_MAX;
}

// requirement.Has(value) for a value that may be absent from the dictionary
static bool req_has_vid(const Dict& D, const Reqs& reqs, int key, int vid) {
    if (key < 0) return true;
    auto it = reqs.m.find(key);
    if (it == reqs.m.end()) return true;  // undefined key: Get() is Exists
    const Req& r = it->second;
    if (vid < 0) return r.complement && !r.has_gt && !r.has_lt;
    return req_has(D, r, vid);
}

static int consolidate_probe_count(const kp_consolidate_input* in) {
    const int n = in->n_candidates;
    if (in->mode == KP_CONSOLIDATE_SINGLE) return n;
    if (n < 2) return 0;
    const int mx = in->max_candidates > 0 ? in->max_candidates : 100;
    return n <= mx ? n - 1 : mx;  // firstNConsolidationOption: mid in [1, max], prefix candidates[0 : mid+1]
}

// The replacement NodeClaim of a REPLACE probe (computeConsolidation's Command.Replacements[0]).
struct Replacement {
    int nodepool = -1;
    int n_held = 0;
    std::vector<int> opts;  // catalog rows, OrderByPrice order
    Reqs reqs;
};

// One SimulateScheduling + computeConsolidation (+ the multi-node filterOutSameInstanceType test).
static void run_probe(const ConsCtx& X, int probe, kp_probe_result& pr, Replacement* rep = nullptr) {
    const kp_consolidate_input* in = X.in;
    const Solver& b = *X.base;
    const int c0 = in->mode == KP_CONSOLIDATE_SINGLE ? probe : 0;
    const int c1 = in->mode == KP_CONSOLIDATE_SINGLE ? probe + 1 : probe + 2;
    pr = kp_probe_result{};
    Solver s(b.D);
    s.R = b.R;
    s.cpu_axis = b.cpu_axis;
    s.mem_axis = b.mem_axis;
    s.hostname_key = b.hostname_key;
    s.host_req = b.host_req;
    s.rid_names = b.rid_names;
    s.rcap = b.rcap;
    s.resv_key = b.resv_key;
    s.resv_on = b.resv_on;
    s.resv_strict = b.resv_strict;
    // the simulation's scheduler relaxes preferences and minValues as provisioning does (PREFERENCE_POLICY /
    // MIN_VALUES_POLICY are controller-wide options; scheduling.md:217-219 "when determining if a pod can be shifted")
    s.relax_next = b.relax_next;
    s.best_effort = b.best_effort;
    s.tp = &b.own_types;
    s.cp = &b.own_classes;
    s.pp = &b.own_pods;
    s.ex_base = &b.own_existing;
    s.tmpls = b.tmpls;
    // SimulateScheduling: state nodes minus the candidates; NewScheduler recomputes NodePool remaining resources over
    // those nodes, i.e. the candidates' capacity returns to their NodePools.
    std::vector<uint8_t> excluded(b.own_existing.size(), 0);
    double cprice = 0;
    bool all_spot = true;
    for (int c = c0; c < c1; c++) {
        const kp_candidate& cd = in->candidates[c];
        excluded[cd.node] = 1;
        cprice += cd.price;  // getCandidatePrices
        if (cd.capacity_type != KP_CT_SPOT) all_spot = false;
        if (cd.capacity && cd.nodepool >= 0)
            for (auto& tm : s.tmpls)
                if (tm.np_index == cd.nodepool)
                    for (int r = 0; r < s.R; r++)
                        if (tm.limit_set[r]) tm.remaining[r] += cd.capacity[r];
    }
    for (int j = 0; j < (int)b.own_existing.size(); j++)
        if (!excluded[j]) s.ex_idx.push_back(j);
    // pods = pending + candidates' reschedulable pods
    for (int i = 0; i < in->n_pending; i++) s.plist.push_back(in->pending[i]);
    const int n_pending = (int)s.plist.size();
    for (int c = c0; c < c1; c++)
        for (int i = 0; i < in->candidates[c].n_pods; i++) s.plist.push_back(in->candidates[c].pods[i]);
    // NewTopology of the simulation: the domain groups, then countDomains over the pods bound in the cluster except
    // the ones this simulation schedules (excludedPods = its candidates' reschedulable pods): the pods of
    // cluster.bound and every other candidate's reschedulable pods on that candidate's node
    if (!b.groups.empty()) {
        s.groups_dg = b.groups_dg;
        s.ident_groups = b.ident_groups;
        s.late_ident = b.late_ident;
        s.cls_birth = b.cls_birth;
        s.n_late = b.n_late;
        s.n_input = b.n_input;
        for (int i = 0; i < in->cluster.n_bound; i++) s.bound_pods.push_back({in->cluster.bound_node[i], in->cluster.bound_class[i]});
        for (int c = 0; c < in->n_candidates; c++) {
            if (c >= c0 && c < c1) continue;
            const kp_candidate& cd = in->candidates[c];
            for (int i = 0; i < cd.n_pods; i++) s.bound_pods.push_back({cd.node, b.own_pods[cd.pods[i]].cls});
        }
        s.new_topology();  // each identity from the first of this simulation's pods that owns it
    }
    pr.n_pods = (int)s.plist.size();
    pr.candidate_price = cprice;

    s.solve();
    s.finalize(in->cluster.max_instance_types);  // Solve(...).TruncateInstanceTypes(MaxInstanceTypes)

    // Results.AllNonPendingPodsScheduled: pending pods may stay pending; a pod placed on an uninitialized existing
    // node is an error (SimulateScheduling)
    bool all = true;
    for (int li = n_pending; li < (int)s.plist.size(); li++) {
        const int r = s.pod_result[li];
        if (r == KP_POD_UNSCHEDULABLE) all = false;
        if (r <= -2 && in->initialized && !in->initialized[-2 - r]) all = false;
    }
    std::vector<int> valid;
    for (int i = 0; i < (int)s.ncs.size(); i++)
        if (s.ncs[i].valid) valid.push_back(i);
    pr.all_scheduled = all ? 1 : 0;
    pr.n_new_nodeclaims = valid.size() < 2 ? (int)valid.size() : 2;
    if (!all) return;
    if (valid.empty()) {
        pr.decision = KP_DECISION_DELETE;
        pr.valid = 1;
        return;
    }
    if (valid.size() != 1) return;  // "we're not going to turn a single node into multiple candidates"
    NodeClaim& nc = s.ncs[valid[0]];
    Reqs reqs = nc.reqs;
    std::vector<int> opts = nc.truncated;  // already OrderByPrice(reqs)
    const int ncand = c1 - c0;
    auto price_filter = [&](const Reqs& rq, double maxp) {  // RemoveInstanceTypeOptionsByPriceAndMinValues / filterByPrice
        std::vector<int> o;
        for (int t : opts)
            if (worst_launch_price(X, t, rq) < maxp) o.push_back(t);
        return o;
    };
    const bool has_spot = req_has_vid(b.D, reqs, X.ct_key, X.v_spot);
    if (all_spot && has_spot) {
        // computeSpotToSpotConsolidation
        if (!in->spot_to_spot) return;
        if (X.ct_key >= 0) reqs.add(b.D, X.spot_req);
        opts = price_filter(reqs, cprice);
        int need = 0;
        if (!s.satisfies_min_values(opts, reqs, &need)) return;
        if (opts.empty()) return;
        if (ncand == 1) {
            if ((int)opts.size() < 15) return;  // MinInstanceTypesForSpotToSpotConsolidation
            const int keep = reqs.has_min_values() ? std::max(15, need) : 15;
            if ((int)opts.size() > keep) opts.resize(keep);
        }
    } else {
        opts = price_filter(reqs, cprice);
        if (!s.satisfies_min_values(opts, reqs)) return;
        if (opts.empty()) return;
        if (has_spot && req_has_vid(b.D, reqs, X.ct_key, X.v_od) && X.ct_key >= 0) reqs.add(b.D, X.spot_req);
    }
    pr.decision = KP_DECISION_REPLACE;
    if (in->mode == KP_CONSOLIDATE_MULTI) {
        // filterOutSameInstanceType: the replacement must be cheaper than the cheapest candidate of a type it offers
        double maxp = DBL_MAX;
        for (int t : opts)
            for (int c = c0; c < c1; c++) {
                const kp_candidate& cd = in->candidates[c];
                if (cd.instance_type == t && cd.price < maxp) maxp = cd.price;
            }
        opts = price_filter(reqs, maxp);
    }
    pr.valid = opts.empty() ? 0 : 1;
    pr.n_replacement_types = (int)opts.size();
    double best = 0;
    for (size_t i = 0; i < opts.size(); i++) {
        const double w = worst_launch_price(X, opts[i], reqs);
        if (i == 0 || w < best) best = w;
    }
    pr.replacement_price = best;
    if (rep) {
        rep->nodepool = s.tmpls[nc.tmpl].np_index;
        rep->n_held = (int)nc.held.size();
        rep->opts = opts;
        rep->reqs = reqs;
    }
}

}  // namespace orc

extern "C" int32_t orc_consolidate_probe_count(const kp_consolidate_input* in) {
    return in ? consolidate_probe_count(in) : 0;
}

static std::atomic<double> g_last_probe_seconds{0.0};

static std::string reqs_text(const orc::Dict& D, const orc::Reqs& reqs);

// Parsed cluster of a consolidation pass, shared read-only by its probes.
struct ConsEnv {
    Dict D;
    Solver base{D};
    ConsCtx X;
};

static kp_status cons_setup(const kp_catalog_view* cat, const kp_consolidate_input* in, const kp_device_opts* opts,
                            ConsEnv& env) {
    if (!cat || !in) return KP_E_INVALID;
    if (in->cluster.min_values_policy != KP_MIN_VALUES_STRICT && in->cluster.min_values_policy != KP_MIN_VALUES_BEST_EFFORT)
        return KP_E_INVALID;
    Dict& D = env.D;
    Solver& base = env.base;
    base.resv_on = true;        // ReservedCapacity gate on; disruption simulations use ReservedOfferingModeFallback
    base.resv_strict = false;
    base.best_effort = in->cluster.min_values_policy == KP_MIN_VALUES_BEST_EFFORT;
    kp_status st = parse_into(base, cat, &in->cluster, opts ? opts->preference_policy : KP_PREFERENCE_RESPECT);
    if (st != KP_OK) return st;
    const int E = (int)base.own_existing.size(), P = (int)base.own_pods.size();
    for (int i = 0; i < in->n_pending; i++)
        if (in->pending[i] < 0 || in->pending[i] >= P) return KP_E_INVALID;
    for (int c = 0; c < in->n_candidates; c++) {
        const kp_candidate& cd = in->candidates[c];
        if (cd.node < 0 || cd.node >= E || cd.n_pods < 0 || (cd.n_pods && !cd.pods) || !(cd.price >= 0)) return KP_E_INVALID;
        for (int i = 0; i < cd.n_pods; i++)
            if (cd.pods[i] < 0 || cd.pods[i] >= P) return KP_E_INVALID;
    }
    ConsCtx& X = env.X;
    X.base = &base;
    X.in = in;
    X.ct_key = D.key("karpenter.sh/capacity-type");
    X.ct_reserved.add(D, new_req(D, X.ct_key, OP_IN, {"reserved"}, false, 0));
    X.ct_spot.add(D, new_req(D, X.ct_key, OP_IN, {"spot"}, false, 0));
    X.ct_od.add(D, new_req(D, X.ct_key, OP_IN, {"on-demand"}, false, 0));
    X.spot_req = new_req(D, X.ct_key, OP_IN, {"spot"}, false, 0);
    X.v_spot = D.value(X.ct_key, "spot");
    X.v_od = D.value(X.ct_key, "on-demand");
    return KP_OK;  // the dictionary is frozen from here on: probes only read it
}

// probes [b0, b1) of X.in's mode over nt threads
static void run_probes(const ConsCtx& X, int b0, int b1, kp_probe_result* results, int nt) {
    std::atomic<int> next{b0};
    auto worker = [&]() {
        for (;;) {
            const int i = next.fetch_add(1);
            if (i >= b1) break;
            run_probe(X, i, results[i - b0]);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; t++) th.emplace_back(worker);
    worker();
    for (auto& t : th) t.join();
}

extern "C" kp_status orc_consolidate_opts(const kp_catalog_view* cat, const kp_consolidate_input* in,
                                          const kp_device_opts* opts, kp_probe_result* results, int32_t cap_results,
                                          int32_t n_threads) {
    if (!cat || !in) return KP_E_INVALID;
    if (in->mode != KP_CONSOLIDATE_SINGLE && in->mode != KP_CONSOLIDATE_MULTI) return KP_E_INVALID;
    auto env = std::make_unique<ConsEnv>();
    kp_status st = cons_setup(cat, in, opts, *env);
    if (st != KP_OK) return st;
    const int np = consolidate_probe_count(in);
    const int b0 = in->probe_begin > 0 ? in->probe_begin : 0;
    const int b1 = in->probe_end > 0 && in->probe_end < np ? in->probe_end : np;
    if (b1 - b0 > cap_results) return KP_E_BUFFER;
    const auto tp0 = std::chrono::steady_clock::now();
    run_probes(env->X, b0, b1, results, n_threads > 1 ? n_threads : 1);
    g_last_probe_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - tp0).count();
    return KP_OK;
}

// The consolidation command (kp_consolidate_command's restatement): MultiNodeConsolidation.firstNConsolidationOption's
// binary search (multinodeconsolidation.go), then SingleNodeConsolidation's first non-no-op candidate
// (singlenodeconsolidation.go), in the disruption controller's method order for KP_CONSOLIDATE_BOTH; a REPLACE carries
// its replacement NodeClaim (options after the price filter / spot-to-spot cut / filterOutSameInstanceType, requirements
// with capacity-type narrowed to spot when priced as spot).
extern "C" kp_status orc_consolidate(const kp_catalog_view* cat, const kp_consolidate_input* in,
                                     kp_probe_result* results, int32_t cap_results, int32_t n_threads) {
    return orc_consolidate_opts(cat, in, nullptr, results, cap_results, n_threads);
}

static kp_status fill_command(ConsEnv& env, kp_consolidate_input& im, int chosen, int probe, const kp_probe_result& row,
                              kp_consolidation_command* out);

extern "C" kp_status orc_consolidate_command_opts(const kp_catalog_view* cat, const kp_consolidate_input* in,
                                                  const kp_device_opts* opts, int32_t mode, kp_consolidation_command* out,
                                                  int32_t n_threads) {
    if (!cat || !in || !out) return KP_E_INVALID;
    if (mode != KP_CONSOLIDATE_SINGLE && mode != KP_CONSOLIDATE_MULTI && mode != KP_CONSOLIDATE_BOTH) return KP_E_INVALID;
    auto env = std::make_unique<ConsEnv>();
    kp_status st = cons_setup(cat, in, opts, *env);
    if (st != KP_OK) return st;
    out->decision = KP_DECISION_NONE;
    out->mode = out->probe = out->nodepool = -1;
    out->first_candidate = out->n_candidates = out->n_type_ids = out->n_reserved = 0;
    out->requirements_needed = 0;
    out->result = kp_probe_result{};
    const int nt = n_threads > 1 ? n_threads : 1;
    kp_consolidate_input im = *in;
    int chosen = -1, probe = -1;
    std::vector<kp_probe_result> rows;
    if (mode != KP_CONSOLIDATE_SINGLE) {
        im.mode = KP_CONSOLIDATE_MULTI;
        env->X.in = &im;
        const int n = consolidate_probe_count(&im);
        rows.assign(std::max(n, 1), kp_probe_result{});
        run_probes(env->X, 0, n, rows.data(), nt);
        // firstNConsolidationOption: mid in [1, max], the prefix candidates[0 : mid+1] is row mid - 1
        if (in->n_candidates >= 2) {
            int lo = 1, hi = in->max_candidates > 0 ? in->max_candidates : 100;
            if (in->n_candidates <= hi) hi = in->n_candidates - 1;
            while (lo <= hi) {
                const int mid = (lo + hi) / 2;
                if (rows[mid - 1].valid) {
                    probe = mid - 1;
                    lo = mid + 1;
                } else {
                    hi = mid - 1;
                }
            }
        }
        if (probe >= 0) chosen = KP_CONSOLIDATE_MULTI;
    }
    if (chosen < 0 && mode != KP_CONSOLIDATE_MULTI) {
        im.mode = KP_CONSOLIDATE_SINGLE;
        env->X.in = &im;
        rows.assign(std::max(in->n_candidates, 1), kp_probe_result{});
        run_probes(env->X, 0, in->n_candidates, rows.data(), nt);
        for (int i = 0; i < in->n_candidates && chosen < 0; i++)
            if (rows[i].decision != KP_DECISION_NONE) {
                chosen = KP_CONSOLIDATE_SINGLE;
                probe = i;
            }
    }
    if (chosen < 0) return KP_OK;
    return fill_command(*env, im, chosen, probe, rows[probe], out);
}

// The command of probe `probe` of mode `chosen` with its row: delete set, and for a REPLACE the replacement NodeClaim
// (the probe re-run with the read-back).
static kp_status fill_command(ConsEnv& env, kp_consolidate_input& im, int chosen, int probe, const kp_probe_result& row,
                              kp_consolidation_command* out) {
    out->mode = chosen;
    out->probe = probe;
    out->first_candidate = chosen == KP_CONSOLIDATE_SINGLE ? probe : 0;
    out->n_candidates = chosen == KP_CONSOLIDATE_SINGLE ? 1 : probe + 2;
    out->result = row;
    out->decision = row.decision;
    if (out->decision != KP_DECISION_REPLACE) return KP_OK;
    im.mode = chosen;
    env.X.in = &im;
    Replacement rep;
    kp_probe_result again{};
    run_probe(env.X, probe, again, &rep);
    out->nodepool = rep.nodepool;
    out->n_reserved = rep.n_held;
    out->n_type_ids = (int)rep.opts.size();
    const std::string txt = reqs_text(env.D, rep.reqs);
    out->requirements_needed = (int64_t)txt.size() + 1;
    bool small = false;
    for (int i = 0; i < out->n_type_ids; i++) {
        if (i < out->cap_type_ids && out->type_ids) out->type_ids[i] = rep.opts[i];
        else small = true;
    }
    if (out->requirements && out->cap_requirements >= (int64_t)txt.size() + 1)
        memcpy(out->requirements, txt.c_str(), txt.size() + 1);
    else
        small = true;
    return small ? KP_E_BUFFER : KP_OK;
}

// kp_consolidate_replacement's restatement: the command of one given probe (its row, and the replacement of a REPLACE).
extern "C" kp_status orc_consolidate_replacement_opts(const kp_catalog_view* cat, const kp_consolidate_input* in,
                                                      const kp_device_opts* opts, int32_t mode, int32_t probe,
                                                      kp_consolidation_command* out) {
    if (!cat || !in || !out) return KP_E_INVALID;
    if (mode != KP_CONSOLIDATE_SINGLE && mode != KP_CONSOLIDATE_MULTI) return KP_E_INVALID;
    auto env = std::make_unique<ConsEnv>();
    kp_status st = cons_setup(cat, in, opts, *env);
    if (st != KP_OK) return st;
    kp_consolidate_input im = *in;
    im.mode = mode;
    if (probe < 0 || probe >= consolidate_probe_count(&im)) return KP_E_INVALID;
    out->decision = KP_DECISION_NONE;
    out->mode = out->probe = out->nodepool = -1;
    out->first_candidate = out->n_candidates = out->n_type_ids = out->n_reserved = 0;
    out->requirements_needed = 0;
    out->result = kp_probe_result{};
    env->X.in = &im;
    kp_probe_result row{};
    run_probe(env->X, probe, row);
    return fill_command(*env, im, mode, probe, row, out);
}

extern "C" kp_status orc_consolidate_command(const kp_catalog_view* cat, const kp_consolidate_input* in, int32_t mode,
                                             kp_consolidation_command* out, int32_t n_threads) {
    return orc_consolidate_command_opts(cat, in, nullptr, mode, out, n_threads);
}

// Wall time of the probe phase of the last orc_consolidate (input parsing excluded): bench.py's CPU baseline.
extern "C" double orc_consolidate_last_probe_seconds(void) { return g_last_probe_seconds; }

// canonical serialization: "key\tcomplement\tgt\tlt\tmin\tv1\x1fv2..." values sorted as strings, keys sorted
static std::string reqs_text(const orc::Dict& D, const orc::Reqs& reqs) {
    std::string s;
    std::vector<std::string> lines;
    for (auto& kv : reqs.m) {
        const Req& r = kv.second;
        std::string l = D.keys[kv.first] + "\t" + (r.complement ? "1" : "0") + "\t" +
                        (r.has_gt ? std::to_string(r.gt) : "-") + "\t" + (r.has_lt ? std::to_string(r.lt) : "-") +
                        "\t" + (r.has_min ? std::to_string(r.min_values) : "-") + "\t";
        std::vector<std::string> vs;
        for (int v : r.values) vs.push_back(D.vals[kv.first][v]);
        std::sort(vs.begin(), vs.end());
        for (size_t i = 0; i < vs.size(); i++) {
            if (i) l += '\x1f';
            l += vs[i];
        }
        lines.push_back(l);
    }
    std::sort(lines.begin(), lines.end());
    for (auto& l : lines) s += l + "\n";
    return s;
}

extern "C" kp_status orc_result_nodeclaim_requirements(const orc_result* res, int32_t nc, char* buf, int64_t cap,
                                                       int64_t* needed) {
    if (!res || nc < 0 || nc >= (int)res->ncs.size()) return KP_E_INVALID;
    const std::string s = reqs_text(res->D, res->ncs[nc].reqs);
    if (needed) *needed = (int64_t)s.size() + 1;
    if ((int64_t)s.size() + 1 > cap) return KP_E_BUFFER;
    memcpy(buf, s.c_str(), s.size() + 1);
    return KP_OK;
}

extern "C" void orc_result_free(orc_result* res) { delete res; }
