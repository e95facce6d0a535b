// ORACLE — test infrastructure only (see oracle/README.md). Never linked into libkpsim.
//
// Launch-time selection, restated on Go-shaped lists from:
//   pkg/providers/instance/instance.go:270-298 filterInstanceTypes (filter chain, ICE on an empty result, Truncate)
//   pkg/providers/instance/filter/filter.go:39-386 (the six filters, literally: slices of types, each with its own
//     offering slice that the offering filters replace)
//   [core] InstanceTypes.OrderByPrice / Truncate / SatisfiesMinValues (recalled)
//   pkg/providers/instance/instance.go:532-546 getCapacityType, :420-467 getOverrides (offering side)
// Go-map iteration (lo.Values at filter.go:115,263) is replaced by input order, as in include/kpsim.h.
#include <algorithm>
#include <cfloat>
#include <cstring>
#include <string>
#include <vector>

#include "orc_api.h"
#include "orc_req.h"

namespace orc {
namespace {

const char* const kCT = "karpenter.sh/capacity-type";
const char* const kZone = "topology.kubernetes.io/zone";
const char* const kResvType = "karpenter.k8s.aws/capacity-reservation-type";
const char* const kSize = "karpenter.k8s.aws/instance-size";

struct Off {
    int row;
    Reqs reqs;
    double price;
    bool available;
    int rcap;
};
struct IT {
    int row;
    std::string name;
    Reqs reqs;
    std::vector<int64_t> cap, alloc;
    std::vector<Off> offs;  // it.Offerings (replaced by the offering filters)
};

struct L {
    Dict D;
    std::vector<std::string> res;
    int kct, kzone, krt, ksize;
    std::string str(int key, const Req& r) const {  // Requirement.Any() for an In requirement, "" otherwise
        if (r.complement || r.values.empty()) return "";
        return D.vals[key][r.values[0]];
    }
    std::string ct(const Off& o) const { return str(kct, o.reqs.get(kct)); }
    std::string zone(const Off& o) const { return str(kzone, o.reqs.get(kzone)); }
    std::string rtype(const Off& o) const { return str(krt, o.reqs.get(krt)); }
    bool has_value(const Reqs& r, int key, const std::string& v) {
        return req_has(D, r.get(key), D.value(key, v));
    }
    // Offerings.Available().Compatible(reqs) over a candidate's current offering list
    std::vector<const Off*> avail_compat(const std::vector<const Off*>& offs, const Reqs& reqs) const {
        std::vector<const Off*> o;
        for (auto* f : offs)
            if (f->available && reqs_compatible(D, reqs, f->reqs, true)) o.push_back(f);
        return o;
    }
};

// One element of the filters' []*InstanceType: the catalog type and its (possibly replaced) offering slice.  Types are
// shared, never copied per request.
struct Cand {
    const IT* it;
    std::vector<const Off*> offs;
};

bool fits(const std::vector<int64_t>& req, const std::vector<int64_t>& alloc) {
    for (size_t r = 0; r < req.size(); r++)
        if (req[r] != 0 && req[r] > alloc[r]) return false;
    return true;
}

}  // namespace
}  // namespace orc

using namespace orc;

extern "C" kp_status orc_launch_select(const kp_catalog_view* cat, int32_t n, const kp_launch_request* requests,
                                       int32_t M, kp_launch_result* results, int32_t* type_ids, int32_t cap_type_ids,
                                       int32_t* override_offerings, int32_t cap_overrides) {
    L X;
    Dict& D = X.D;
    const int T = cat->n_types, R = cat->n_resources;
    for (int r = 0; r < R; r++) X.res.emplace_back(cat->resource_names[r]);
    X.kct = D.key(kCT);
    X.kzone = D.key(kZone);
    X.krt = D.key(kResvType);
    X.ksize = D.key(kSize);
    std::vector<IT> all(T);
    for (int t = 0; t < T; t++) {
        IT& it = all[t];
        it.row = t;
        it.name = cat->type_names[t];
        it.cap.assign(cat->capacity + (size_t)t * R, cat->capacity + (size_t)(t + 1) * R);
        it.alloc.assign(cat->allocatable + (size_t)t * R, cat->allocatable + (size_t)(t + 1) * R);
        for (int k = 0; k < cat->n_label_keys; k++) {
            const int st = cat->label_state[(size_t)t * cat->n_label_keys + k];
            if (st == KP_LABEL_ABSENT) continue;
            const int key = D.key(normalize_label(cat->label_keys[k]));
            std::vector<std::string> vs;
            if (st == KP_LABEL_IN)
                for (int i = cat->label_offsets[(size_t)t * cat->n_label_keys + k];
                     i < cat->label_offsets[(size_t)t * cat->n_label_keys + k + 1]; i++)
                    vs.emplace_back(cat->label_values[i]);
            it.reqs.add(D, new_req(D, key, vs.empty() ? OP_DNE : OP_IN, vs, false, 0));
        }
    }
    for (int o = 0; o < cat->n_offerings; o++) {
        Off f;
        f.row = o;
        f.price = cat->offering_price[o];
        f.available = cat->offering_available[o] != 0;
        f.rcap = cat->offering_reservation_capacity ? cat->offering_reservation_capacity[o] : 0;
        for (int k = 0; k < cat->n_offering_keys; k++) {
            const int st = cat->offering_label_state[(size_t)o * cat->n_offering_keys + k];
            if (st == KP_LABEL_ABSENT) continue;
            const int key = D.key(normalize_label(cat->offering_keys[k]));
            if (st == KP_LABEL_DOES_NOT_EXIST) f.reqs.add(D, new_req(D, key, OP_DNE, {}, false, 0));
            else f.reqs.add(D, new_req(D, key, OP_IN, {cat->offering_label_values[(size_t)o * cat->n_offering_keys + k]}, false, 0));
        }
        all[cat->offering_type[o]].offs.push_back(f);
    }
    const char* accel[] = {"aws.amazon.com/neuron", "aws.amazon.com/neuroncore", "amd.com/gpu", "nvidia.com/gpu",
                           "habana.ai/gaudi"};
    int tpos = 0, opos = 0;
    bool short_buf = false;
    for (int i = 0; i < n; i++) {
        const kp_launch_request& lr = requests[i];
        Reqs reqs;  // NewNodeSelectorRequirementsWithMinValues
        for (int j = 0; j < lr.n_requirements; j++) {
            const kp_requirement& r = lr.requirements[j];
            std::vector<std::string> vs;
            for (int v = 0; v < r.n_values; v++) vs.emplace_back(r.values[v] ? r.values[v] : "");
            reqs.add(D, new_req(D, D.key(normalize_label(r.key)), (Op)r.op, vs, r.min_values >= 0, r.min_values));
        }
        std::vector<int64_t> rq(R, 0);
        if (lr.requests) rq.assign(lr.requests, lr.requests + R);
        kp_launch_result& res = results[i];
        memset(&res, 0, sizeof(res));
        res.failed_filter = -1;
        res.capacity_type = KP_CT_ON_DEMAND;
        res.type_offset = tpos;
        res.override_offset = opos;
        const bool has_min = reqs.has_min_values();
        const bool has_reserved = X.has_value(reqs, X.kct, "reserved");
        std::vector<Cand> its;
        auto ice = [&](int f) {
            res.status = KP_E_INSUFFICIENT_CAPACITY;
            res.failed_filter = f;
        };
        // CompatibleAvailableFilter (filter.go:51-64)
        {
            for (auto& it : all) {
                if (!reqs_compatible(D, reqs, it.reqs, true)) continue;
                if (!fits(rq, it.alloc)) continue;
                bool any = false;
                for (auto& f : it.offs)
                    if (f.available && reqs_compatible(D, reqs, f.reqs, true)) {
                        any = true;
                        break;
                    }
                if (!any) continue;
                Cand c{&it, {}};
                for (auto& f : it.offs) c.offs.push_back(&f);
                its.push_back(std::move(c));
            }
            res.rejected[0] = (int)(all.size() - its.size());
            if (its.empty()) ice(KP_FILTER_COMPATIBLE_AVAILABLE);
        }
        // CapacityReservationTypeFilter (filter.go:83-157)
        if (res.status == KP_OK && has_reserved) {
            double cheapest[2] = {DBL_MAX, DBL_MAX};
            std::vector<int> member[2];
            for (size_t x = 0; x < its.size(); x++) {
                bool in[2] = {false, false};
                for (auto* o : X.avail_compat(its[x].offs, reqs)) {
                    if (X.ct(*o) != "reserved") continue;
                    const std::string t = X.rtype(*o);
                    const int p = t == "default" ? 0 : (t == "capacity-block" ? 1 : -1);
                    if (p < 0) return KP_E_INVALID;  // filter.go:148 panics
                    if (cheapest[p] > o->price) cheapest[p] = o->price;
                    in[p] = true;
                }
                for (int p = 0; p < 2; p++)
                    if (in[p]) member[p].push_back((int)x);
            }
            const int sel = cheapest[1] < cheapest[0] ? 1 : 0;  // lo.MinBy: price, then priority default < capacity-block
            if (!member[sel].empty()) {
                std::vector<Cand> kept;
                for (int x : member[sel]) {
                    Cand c{its[x].it, {}};
                    for (auto* f : its[x].offs)
                        if (X.ct(*f) == "reserved" && X.rtype(*f) == (sel ? "capacity-block" : "default")) c.offs.push_back(f);
                    kept.push_back(std::move(c));
                }
                res.rejected[1] = (int)(its.size() - kept.size());
                its.swap(kept);
            }
        }
        // CapacityBlockFilter (filter.go:173-221)
        if (res.status == KP_OK && has_reserved) {
            bool should = false, decided = false;
            for (auto& c : its) {
                for (auto* f : c.offs) {
                    if (!f->reqs.has(X.krt)) continue;
                    should = X.rtype(*f) == "capacity-block";
                    decided = true;
                    break;
                }
                if (decided) break;
            }
            if (should) {
                int sel = -1;
                const Off* selo = nullptr;
                for (size_t x = 0; x < its.size(); x++) {
                    const Off* so = nullptr;
                    for (auto* f : its[x].offs) {
                        if (X.ct(*f) != "reserved" || X.rtype(*f) != "capacity-block") continue;
                        if (!so || so->price > f->price) so = f;
                    }
                    if (so && (sel < 0 || selo->price > so->price)) {
                        selo = so;
                        sel = (int)x;
                    }
                }
                Cand c{its[sel].it, {selo}};
                res.rejected[2] = (int)its.size() - 1;
                its.clear();
                its.push_back(std::move(c));
            }
        }
        // ReservedOfferingFilter (filter.go:240-270)
        if (res.status == KP_OK && has_reserved) {
            std::vector<Cand> remaining;
            for (auto& c : its) {
                std::vector<std::string> zones;
                std::vector<const Off*> zo;
                for (auto* o : X.avail_compat(c.offs, reqs)) {
                    if (X.ct(*o) != "reserved") continue;
                    const std::string z = X.zone(*o);
                    size_t k = 0;
                    while (k < zones.size() && zones[k] != z) k++;
                    if (k == zones.size()) {
                        zones.push_back(z);
                        zo.push_back(o);
                    } else if (o->rcap > zo[k]->rcap) {
                        zo[k] = o;
                    }
                }
                if (zo.empty()) continue;
                std::sort(zo.begin(), zo.end(), [](const Off* a, const Off* b) { return a->row < b->row; });
                remaining.push_back(Cand{c.it, zo});
            }
            if (!remaining.empty()) {
                res.rejected[3] = (int)(its.size() - remaining.size());
                its.swap(remaining);
            }
        }
        // ExoticInstanceTypeFilter (filter.go:289-318)
        if (res.status == KP_OK && !has_min) {
            std::vector<Cand> generic;
            for (auto& c : its) {
                bool exotic = false;
                const Req sz = c.it->reqs.get(X.ksize);
                if (!sz.complement)
                    for (int v : sz.values)
                        if (D.vals[X.ksize][v].find("metal") != std::string::npos) exotic = true;
                for (int r = 0; r < R; r++)
                    for (auto* a : accel)
                        if (X.res[r] == a && c.it->cap[r] != 0) exotic = true;
                if (!exotic) generic.push_back(c);
            }
            if (!generic.empty()) {
                res.rejected[4] = (int)(its.size() - generic.size());
                its.swap(generic);
            }
        }
        // SpotInstanceFilter (filter.go:339-386)
        if (res.status == KP_OK && !has_min && X.has_value(reqs, X.kct, "on-demand") && X.has_value(reqs, X.kct, "spot")) {
            double cod = DBL_MAX;
            bool has_spot = false, has_od = false;
            for (auto& c : its)
                for (auto* o : X.avail_compat(c.offs, reqs)) {
                    const std::string ctv = X.ct(*o);
                    if (ctv == "on-demand") {
                        has_od = true;
                        if (o->price < cod) cod = o->price;
                    } else if (ctv == "spot") {
                        has_spot = true;
                    }
                }
            if (has_od && has_spot) {
                std::vector<Cand> kept;
                for (auto& c : its) {
                    bool keep = false, decided = false, spot = false;
                    for (auto* o : X.avail_compat(c.offs, reqs)) {
                        const std::string ctv = X.ct(*o);
                        if (ctv == "reserved") {
                            keep = decided = true;
                            break;
                        }
                        if (ctv == "spot") {
                            spot = true;
                            if (o->price <= cod) {
                                keep = decided = true;
                                break;
                            }
                        }
                    }
                    if (!decided) keep = !spot;
                    if (keep) kept.push_back(c);
                }
                res.rejected[5] = (int)(its.size() - kept.size());
                its.swap(kept);
                if (its.empty()) ice(KP_FILTER_SPOT);
            }
        }
        if (res.status != KP_OK) continue;
        res.n_options = (int)its.size();
        // Truncate(reqs, M): OrderByPrice then SatisfiesMinValues
        std::vector<std::pair<double, int>> key;
        for (size_t x = 0; x < its.size(); x++) {
            double p = DBL_MAX;
            for (auto* o : X.avail_compat(its[x].offs, reqs))
                if (o->price < p) p = o->price;
            key.emplace_back(p, (int)x);
        }
        std::sort(key.begin(), key.end(), [&](const std::pair<double, int>& a, const std::pair<double, int>& b) {
            if (a.first != b.first) return a.first < b.first;
            if (its[a.second].it->name != its[b.second].it->name) return its[a.second].it->name < its[b.second].it->name;
            return its[a.second].it->row < its[b.second].it->row;
        });
        if ((int)key.size() > M) key.resize(M);
        if (has_min) {
            for (auto& kv : reqs.m) {
                if (!kv.second.has_min) continue;
                std::vector<int> seen;
                for (auto& k : key) {
                    const Req r = its[k.second].it->reqs.get(kv.first);
                    if (r.complement) continue;
                    for (int v : r.values)
                        if (std::find(seen.begin(), seen.end(), v) == seen.end()) seen.push_back(v);
                }
                if ((int)seen.size() < kv.second.min_values) res.status = KP_E_CREATE;
            }
            if (res.status != KP_OK) continue;
        }
        // getCapacityType (instance.go:532-546)
        int ct = KP_CT_ON_DEMAND;
        const char* names[3] = {"on-demand", "spot", "reserved"};
        for (int c : {KP_CT_RESERVED, KP_CT_SPOT}) {
            if (!X.has_value(reqs, X.kct, names[c])) continue;
            Reqs r2 = reqs;
            r2.m[X.kct] = new_req(D, X.kct, OP_IN, {names[c]}, false, 0);
            bool any = false;
            for (auto& k : key)
                if (!X.avail_compat(its[k.second].offs, r2).empty()) {
                    any = true;
                    break;
                }
            if (any) {
                ct = c;
                break;
            }
        }
        res.capacity_type = ct;
        // kwok CreateFleet (kwok/ec2/ec2.go:432-461, kwok/strategy/strategy.go:45-60): lo.MinBy over the overrides in
        // order, score = SpotPrice(type, zone) for a spot fleet else OnDemandPrice(type), MaxFloat64 without a price;
        // MinBy's comparison holds when the running minimum's score is 0 (lo.IsEmpty) or item < minimum with item != 0
        res.fleet_pick = -1;
        double best_score = 0;
        auto fleet_score = [&](const Off& o, const IT& it) {
            for (auto& f : it.offs) {
                if (ct == KP_CT_SPOT) {
                    if (X.ct(f) == "spot" && X.zone(f) == X.zone(o)) return f.price;
                } else if (X.ct(f) == "on-demand") {
                    return f.price;
                }
            }
            return DBL_MAX;
        };
        Reqs r3 = reqs;
        r3.m[X.kct] = new_req(D, X.kct, OP_IN, {names[ct]}, false, 0);
        res.n_types = (int)key.size();
        for (auto& k : key) {
            if (type_ids && tpos < cap_type_ids) type_ids[tpos] = its[k.second].it->row;
            else short_buf = true;
            tpos++;
            for (auto* o : X.avail_compat(its[k.second].offs, r3)) {
                const double sc = fleet_score(*o, *its[k.second].it);
                if (res.fleet_pick < 0 || best_score == 0.0 || (sc != 0.0 && sc < best_score)) {
                    res.fleet_pick = o->row;
                    best_score = sc;
                }
                if (override_offerings && opos < cap_overrides) override_offerings[opos] = o->row;
                else short_buf = true;
                opos++;
                res.n_overrides++;
            }
        }
    }
    return short_buf ? KP_E_BUFFER : KP_OK;
}
