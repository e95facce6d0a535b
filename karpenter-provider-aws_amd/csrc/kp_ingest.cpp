// kp_ingest.cpp — catalog ingestion: raw EC2 instance-type data + EC2NodeClass → the
// `[]*cloudprovider.InstanceType` snapshot as a kp_catalog_view (host code; the catalog is built once per cache miss,
// ~1k types, then uploaded with kp_catalog_upload).
//
// Restated from the reference (file:line per function below):
//   pkg/providers/instancetype/types.go:123-155  NewInstanceType
//   pkg/providers/instancetype/types.go:158-299  computeRequirements
//   pkg/providers/instancetype/types.go:320-605  computeCapacity, memory, ephemeralStorage, pods, ENILimitedPods,
//                                                kubeReservedResources, systemReservedResources, evictionThreshold
//   pkg/providers/amifamily/{resolver,al2,al2023,bottlerocket,windows,custom}.go  feature flags, default block devices
//   pkg/providers/instancetype/offering/offering.go:103-196  createOfferings
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "../../include/kpsim.h"

namespace {

const char* const kResources[KP_CATALOG_R] = {
    "cpu", "memory", "ephemeral-storage", "pods", "vpc.amazonaws.com/pod-eni", "nvidia.com/gpu", "amd.com/gpu",
    "aws.amazon.com/neuron", "aws.amazon.com/neuroncore", "habana.ai/gaudi", "vpc.amazonaws.com/efa",
    "vpc.amazonaws.com/PrivateIPv4Address"};
enum { R_CPU = 0, R_MEM, R_EPH, R_PODS, R_PODENI, R_NVIDIA, R_AMD, R_NEURON, R_NEURONCORE, R_GAUDI, R_EFA, R_PRIVIP };

const char* const AWS = "karpenter.k8s.aws/";
const std::string K_ITYPE = "node.kubernetes.io/instance-type", K_ARCH = "kubernetes.io/arch", K_OS = "kubernetes.io/os",
                  K_ZONE = "topology.kubernetes.io/zone", K_REGION = "topology.kubernetes.io/region",
                  K_WINBUILD = "node.kubernetes.io/windows-build", K_CT = "karpenter.sh/capacity-type",
                  K_ZONEID = "topology.k8s.aws/zone-id", K_RESVID = "karpenter.k8s.aws/capacity-reservation-id",
                  K_RESVTYPE = "karpenter.k8s.aws/capacity-reservation-type";
std::string aws(const char* s) { return std::string(AWS) + s; }

// the keys computeRequirements always sets (types.go:181-234), in a fixed order, then zone-id (added when the
// NodeClass maps an available zone, :236-244)
std::vector<std::string> type_keys() {
    return {K_ITYPE, K_ARCH, K_OS, K_ZONE, K_REGION, K_WINBUILD, K_CT,
            aws("instance-cpu"), aws("instance-cpu-manufacturer"), aws("instance-cpu-sustained-clock-speed-mhz"),
            aws("instance-memory"), aws("instance-ebs-bandwidth"), aws("instance-network-bandwidth"),
            aws("instance-category"), aws("instance-capacity-flex"), aws("instance-family"),
            aws("instance-generation"), aws("instance-local-nvme"), aws("instance-size"), aws("instance-gpu-name"),
            aws("instance-gpu-manufacturer"), aws("instance-gpu-count"), aws("instance-gpu-memory"),
            aws("instance-accelerator-name"), aws("instance-accelerator-manufacturer"),
            aws("instance-accelerator-count"), aws("instance-hypervisor"),
            aws("instance-encryption-in-transit-supported"), K_RESVID, K_RESVTYPE, K_ZONEID};
}
const char* const kOfferingKeys[5] = {"karpenter.sh/capacity-type", "topology.kubernetes.io/zone",
                                      "karpenter.k8s.aws/capacity-reservation-id",
                                      "karpenter.k8s.aws/capacity-reservation-type", "topology.k8s.aws/zone-id"};

struct Flags {  // amifamily FeatureFlags (resolver.go:113-119, bottlerocket.go:126-131, windows.go:101-107)
    bool eni_mem, ppc, evsoft, eni_pods;
};
Flags flags_of(int fam) {
    if (fam == KP_AMI_BOTTLEROCKET) return {false, false, false, true};
    if (fam == KP_AMI_WINDOWS2019 || fam == KP_AMI_WINDOWS2022) return {false, true, true, false};
    return {true, true, true, true};
}
bool windows(int fam) { return fam == KP_AMI_WINDOWS2019 || fam == KP_AMI_WINDOWS2022; }

std::string lower_kabob(const char* s) {  // types.go:586-588
    std::string o = s ? s : "";
    for (char& c : o) {
        if (c == ' ') c = '-';
        else if (c >= 'A' && c <= 'Z') c = (char)(c - 'A' + 'a');
    }
    return o;
}

// resource.MustParse(s).MilliValue() (rounded up, as Quantity does): decimal mantissa with an optional decimal-SI,
// binary-SI or decimal-exponent suffix.  Returns false on a malformed quantity.
bool quantity_milli(const char* s, int64_t* out) {
    if (!s) return false;
    const char* p = s;
    bool neg = false;
    if (*p == '+' || *p == '-') neg = *p++ == '-';
    __int128 num = 0, den = 1;
    bool digits = false, dot = false;
    for (; (*p >= '0' && *p <= '9') || *p == '.'; p++) {
        if (*p == '.') {
            if (dot) return false;
            dot = true;
            continue;
        }
        digits = true;
        if (num > ((__int128)1 << 100)) return false;
        num = num * 10 + (*p - '0');
        if (dot) den *= 10;
    }
    if (!digits) return false;
    const std::string suf = p;
    __int128 mul = 1, div = 1;
    static const std::map<std::string, std::pair<int, int>> si = {  // (power of 10, power of 2)
        {"", {0, 0}},  {"n", {-9, 0}}, {"u", {-6, 0}}, {"m", {-3, 0}}, {"k", {3, 0}},  {"M", {6, 0}},
        {"G", {9, 0}}, {"T", {12, 0}}, {"P", {15, 0}}, {"E", {18, 0}}, {"Ki", {0, 10}}, {"Mi", {0, 20}},
        {"Gi", {0, 30}}, {"Ti", {0, 40}}, {"Pi", {0, 50}}, {"Ei", {0, 60}}};
    int e10 = 0, e2 = 0;
    auto it = si.find(suf);
    if (it != si.end()) {
        e10 = it->second.first;
        e2 = it->second.second;
    } else if (suf[0] == 'e' || suf[0] == 'E') {  // decimal exponent: 1e3, 1.5E-3, 1e+09
        const char* q = suf.c_str() + 1;
        bool eneg = false;
        if (*q == '+' || *q == '-') eneg = *q++ == '-';
        if (!*q) return false;
        for (; *q; q++) {
            if (*q < '0' || *q > '9' || e10 > 100) return false;
            e10 = e10 * 10 + (*q - '0');
        }
        if (eneg) e10 = -e10;
    } else {
        return false;
    }
    e10 += 3;  // milli
    if (e10 > 30 || e10 < -30) return false;
    for (int i = 0; i < e10; i++) mul *= 10;
    for (int i = 0; i < -e10; i++) div *= 10;
    mul <<= e2;
    const __int128 a = num * mul, b = den * div;
    __int128 v = a / b;
    if (!neg && a % b) v += 1;  // round up (toward +inf)
    if (neg) v = -v;
    if (v > INT64_MAX || v < INT64_MIN) return false;
    *out = (int64_t)v;
    return true;
}

int64_t ceil_div_1000(int64_t milli) { return milli >= 0 ? (milli + 999) / 1000 : -((-milli) / 1000); }

struct Built {
    std::string name;
    std::map<std::string, std::vector<std::string>> labels;  // key -> values (empty: DoesNotExist)
    std::set<std::string> absent;                            // keys not set (zone-id without a mapped zone)
    int64_t cap[KP_CATALOG_R] = {};
    int64_t ovh[KP_CATALOG_R] = {};
};

struct Err {
    std::string msg;
};

int64_t eni_limited_pods(const kp_ec2_instance_type& in, int reserved) {  // types.go:445-459
    const int ifaces = in.n_network_cards > 0 ? in.card_max_interfaces[in.default_card] : in.max_network_interfaces;
    const int64_t usable = std::max<int64_t>((int64_t)ifaces - reserved, 0);
    if (usable == 0) return 0;
    return usable * ((int64_t)in.ipv4_per_interface - 1) + 2;
}

int64_t pods_of(const kp_ec2_instance_type& in, const kp_nodeclass_view& nc, const Flags& f) {  // types.go:562-578
    int64_t count;
    if (nc.max_pods >= 0) count = nc.max_pods;
    else if (f.eni_pods) count = eni_limited_pods(in, nc.reserved_enis);
    else count = 110;
    if (nc.pods_per_core > 0 && f.ppc) count = std::min<int64_t>((int64_t)nc.pods_per_core * in.default_vcpus, count);
    return count;
}

int64_t memory_bytes(const kp_ec2_instance_type& in, const kp_nodeclass_view& nc) {  // types.go:344-354
    int64_t mib = in.memory_mib;
    if (in.n_architectures > 0 && in.architectures[0] && !strcmp(in.architectures[0], "arm64")) mib -= 64;
    const int64_t mem = mib * 1024 * 1024;
    const int64_t over = (int64_t)std::ceil((double)mem * nc.vm_memory_overhead_percent / 1024 / 1024);
    return mem - over * 1024 * 1024;
}

// ephemeralStorage (types.go:357-392) in milli; AMI default block devices (resolver.go:40-43 DefaultEBS 20Gi,
// al2023.go / al2.go /dev/xvda, bottlerocket.go:95-112 /dev/xvdb, windows.go:88-99 /dev/sda1 50Gi, custom.go none)
int64_t ephemeral_milli(const kp_ec2_instance_type& in, const kp_nodeclass_view& nc) {
    const int64_t gi = (int64_t)1 << 30;
    if (nc.instance_store_raid0 && in.instance_storage_gb >= 0) return in.instance_storage_gb * 1000000000LL * 1000;
    const int fam = nc.ami_family;
    const char* eph_dev = fam == KP_AMI_BOTTLEROCKET ? "/dev/xvdb" : windows(fam) ? "/dev/sda1"
                          : fam == KP_AMI_CUSTOM     ? nullptr
                                                     : "/dev/xvda";
    const int64_t def_size = windows(fam) ? 50 * gi : 20 * gi;
    auto size_of = [&](const kp_block_device_mapping& b, int64_t* m) -> bool {
        if (!b.volume_size) return false;
        if (!quantity_milli(b.volume_size, m)) throw Err{std::string("malformed volume size ") + b.volume_size};
        return true;
    };
    if (nc.n_block_device_mappings > 0) {
        const kp_block_device_mapping* bdm = nc.block_device_mappings;
        for (int i = 0; i < nc.n_block_device_mappings; i++) {
            if (bdm[i].root_volume) {
                int64_t m;
                if (size_of(bdm[i], &m)) return m;
                break;  // lo.Find: the first root volume, whose size is nil
            }
        }
        if (fam == KP_AMI_CUSTOM) {
            int64_t m;
            return size_of(bdm[nc.n_block_device_mappings - 1], &m) ? m : 20 * gi * 1000;
        }
        for (int i = 0; i < nc.n_block_device_mappings; i++) {
            if (bdm[i].device_name && eph_dev && !strcmp(bdm[i].device_name, eph_dev)) {
                int64_t m;
                if (size_of(bdm[i], &m)) return m;
                break;
            }
        }
    }
    if (eph_dev) return def_size * 1000;  // the AMI family's ephemeral block device default
    return 20 * gi * 1000;
}

int resource_index(const char* name) {
    for (int r = 0; r < KP_CATALOG_R; r++)
        if (name && !strcmp(name, kResources[r])) return r;
    return -1;
}

// evictionThreshold's computeEvictionSignal (types.go:593-615) on a capacity in bytes; returns milli
int64_t eviction_signal(int64_t capacity_bytes, const char* v) {
    const size_t n = strlen(v);
    if (n > 0 && v[n - 1] == '%') {
        const std::string num(v, n - 1);
        char* end = nullptr;
        double p = strtod(num.c_str(), &end);
        if (end == num.c_str() || *end) throw Err{std::string("malformed percentage ") + v};
        if (p == 100) p = 0;  // 100% disables the threshold
        const double x = std::ceil((double)capacity_bytes / 100 * p);
        return (int64_t)x * 1000;
    }
    int64_t m;
    if (!quantity_milli(v, &m)) throw Err{std::string("malformed quantity ") + v};
    return m;
}

Built build_type(const kp_ec2_instance_type& in, const kp_nodeclass_view& nc, const std::vector<std::string>& off_zones) {
    if (!in.name) throw Err{"instance type without a name"};
    Built b;
    b.name = in.name;
    const Flags f = flags_of(nc.ami_family);
    const int fam = nc.ami_family;
    // ---- computeRequirements (types.go:158-299) ----
    std::vector<const kp_capacity_reservation*> crs;  // instancetype.go:116-118: the type's reservations
    for (int i = 0; i < nc.n_capacity_reservations; i++) {
        const kp_capacity_reservation& cr = nc.capacity_reservations[i];
        if (cr.instance_type && !strcmp(cr.instance_type, in.name)) crs.push_back(&cr);
    }
    std::vector<std::string> cts;
    for (int i = 0; i < in.n_usage_classes; i++) {
        const char* u = in.usage_classes[i];
        if (u && (!strcmp(u, "on-demand") || !strcmp(u, "spot"))) cts.push_back(u);
    }
    if (!crs.empty()) cts.push_back("reserved");
    std::set<std::string> subnet_zones;
    for (int i = 0; i < nc.n_zones; i++)
        if (nc.zones[i].zone) subnet_zones.insert(nc.zones[i].zone);
    std::set<std::string> avail;
    for (const auto& z : off_zones)
        if (subnet_zones.count(z)) avail.insert(z);
    std::string arch;  // getArchitecture (types.go:310-317): first architecture with a kube name
    bool have_arch = false;
    for (int i = 0; i < in.n_architectures && !have_arch; i++) {
        const char* a = in.architectures[i];
        if (a && !strcmp(a, "x86_64")) arch = "amd64", have_arch = true;
        else if (a && !strcmp(a, "arm64")) arch = "arm64", have_arch = true;
    }
    if (!have_arch) {  // fmt.Sprint of the slice, as the reference prints it
        arch = "[";
        for (int i = 0; i < in.n_architectures; i++) arch += std::string(i ? " " : "") + (in.architectures[i] ? in.architectures[i] : "");
        arch += "]";
    }
    auto& L = b.labels;
    for (const auto& k : type_keys()) L[k] = {};
    L[K_ITYPE] = {in.name};
    L[K_ARCH] = {arch};
    if (windows(fam)) L[K_OS] = arch == "amd64" ? std::vector<std::string>{"windows"} : std::vector<std::string>{};
    else L[K_OS] = {"linux"};
    L[K_ZONE] = std::vector<std::string>(avail.begin(), avail.end());
    L[K_REGION] = {nc.region ? nc.region : ""};
    L[K_CT] = cts;
    L[aws("instance-cpu")] = {std::to_string(in.default_vcpus)};
    L[aws("instance-memory")] = {std::to_string(in.memory_mib)};
    L[aws("instance-hypervisor")] = {in.hypervisor ? in.hypervisor : ""};
    L[aws("instance-encryption-in-transit-supported")] = {in.encryption_in_transit ? "true" : "false"};
    {
        std::set<std::string> ids;
        for (int i = 0; i < nc.n_zones; i++)
            if (nc.zones[i].zone && avail.count(nc.zones[i].zone)) ids.insert(nc.zones[i].zone_id ? nc.zones[i].zone_id : "");
        if (!ids.empty()) L[K_ZONEID] = std::vector<std::string>(ids.begin(), ids.end());
        else b.absent.insert(K_ZONEID);
    }
    if (!crs.empty()) {
        std::set<std::string> ids, types;
        for (auto* cr : crs) {
            ids.insert(cr->id ? cr->id : "");
            types.insert(cr->reservation_type ? cr->reservation_type : "");
        }
        L[K_RESVID] = std::vector<std::string>(ids.begin(), ids.end());
        L[K_RESVTYPE] = std::vector<std::string>(types.begin(), types.end());
    }
    {  // instanceTypeScheme (types.go:49): (^[a-z]+)(\-[0-9]+tb)?([0-9]+).*\.
        const std::string s = in.name;
        size_t i = 0;
        while (i < s.size() && s[i] >= 'a' && s[i] <= 'z') i++;
        if (i > 0) {
            const std::string cat = s.substr(0, i);
            size_t j = i;
            if (j < s.size() && s[j] == '-') {  // optional -<n>tb
                size_t k = j + 1;
                while (k < s.size() && isdigit((unsigned char)s[k])) k++;
                if (k > j + 1 && s.compare(k, 2, "tb") == 0) j = k + 2;
            }
            size_t g = j;
            while (g < s.size() && isdigit((unsigned char)s[g])) g++;
            if (g > j && s.find('.', g) != std::string::npos) {
                L[aws("instance-category")] = {cat};
                L[aws("instance-generation")] = {s.substr(j, g - j)};
            }
        }
        std::vector<std::string> parts;
        size_t st = 0;
        for (;;) {
            const size_t d = s.find('.', st);
            parts.push_back(s.substr(st, d == std::string::npos ? std::string::npos : d - st));
            if (d == std::string::npos) break;
            st = d + 1;
        }
        if (parts.size() == 2) {
            L[aws("instance-family")] = {parts[0]};
            L[aws("instance-size")] = {parts[1]};
        }
        L[aws("instance-capacity-flex")] = {parts[0].find("-flex") != std::string::npos ? "true" : "false"};
    }
    if (in.instance_storage_gb >= 0 && !(in.nvme_support && !strcmp(in.nvme_support, "unsupported")))
        L[aws("instance-local-nvme")] = {std::to_string(in.instance_storage_gb)};
    if (in.network_bandwidth_mbps >= 0) L[aws("instance-network-bandwidth")] = {std::to_string(in.network_bandwidth_mbps)};
    if (in.n_gpus == 1) {
        const kp_ec2_device& g = in.gpus[0];
        L[aws("instance-gpu-name")] = {lower_kabob(g.name)};
        L[aws("instance-gpu-manufacturer")] = {lower_kabob(g.manufacturer)};
        L[aws("instance-gpu-count")] = {std::to_string(g.count)};
        L[aws("instance-gpu-memory")] = {std::to_string(g.memory_mib)};
    }
    if (in.n_accelerators == 1 && in.n_neuron < 0) {
        const kp_ec2_device& a = in.accelerators[0];
        L[aws("instance-accelerator-name")] = {lower_kabob(a.name)};
        L[aws("instance-accelerator-manufacturer")] = {lower_kabob(a.manufacturer)};
        L[aws("instance-accelerator-count")] = {std::to_string(a.count)};
    }
    if (in.n_neuron == 1) {
        const kp_ec2_device& d = in.neuron[0];
        L[aws("instance-accelerator-name")] = {lower_kabob(d.name)};
        L[aws("instance-accelerator-manufacturer")] = {"aws"};
        L[aws("instance-accelerator-count")] = {std::to_string(d.count)};
    }
    if (fam == KP_AMI_WINDOWS2019) L[K_WINBUILD] = {"10.0.17763"};  // pkg/apis/v1/labels.go:112-113
    if (fam == KP_AMI_WINDOWS2022) L[K_WINBUILD] = {"10.0.20348"};
    if (in.has_processor_info) {
        L[aws("instance-cpu-manufacturer")] = {lower_kabob(in.cpu_manufacturer)};
        const double ghz = std::isnan(in.sustained_clock_ghz) ? 0.0 : in.sustained_clock_ghz;
        L[aws("instance-cpu-sustained-clock-speed-mhz")] = {std::to_string((long long)std::round(ghz * 1000))};
    }
    if (in.ebs_max_bandwidth_mbps >= 0 && in.ebs_optimized_support && !strcmp(in.ebs_optimized_support, "default"))
        L[aws("instance-ebs-bandwidth")] = {std::to_string(in.ebs_max_bandwidth_mbps)};

    // ---- computeCapacity (types.go:320-338) ----
    int64_t* cap = b.cap;
    cap[R_CPU] = (int64_t)in.default_vcpus * 1000;
    const int64_t mem = memory_bytes(in, nc);
    cap[R_MEM] = mem * 1000;
    const int64_t eph_m = ephemeral_milli(in, nc);
    cap[R_EPH] = eph_m;
    const int64_t pods = pods_of(in, nc, f);
    cap[R_PODS] = pods * 1000;
    cap[R_PODENI] = (in.has_vpc_limits && in.vpc_trunking) ? (int64_t)in.vpc_branch_interface * 1000 : 0;
    for (int i = 0; i < in.n_gpus; i++) {
        const char* m = in.gpus[i].manufacturer;
        if (!m) continue;
        if (!strcmp(m, "NVIDIA")) cap[R_NVIDIA] += (int64_t)in.gpus[i].count * 1000;
        else if (!strcmp(m, "AMD")) cap[R_AMD] += (int64_t)in.gpus[i].count * 1000;
        else if (!strcmp(m, "Habana")) cap[R_GAUDI] += (int64_t)in.gpus[i].count * 1000;
    }
    if (in.n_neuron > 0) {
        for (int i = 0; i < in.n_neuron; i++) cap[R_NEURON] += (int64_t)in.neuron[i].count * 1000;
        cap[R_NEURONCORE] = (int64_t)in.neuron[0].count * in.neuron[0].cores * 1000;
    }
    cap[R_EFA] = (int64_t)in.efa_max * 1000;
    // PrivateIPv4Address for types compatible with os In [windows] (types.go:151-153, privateIPv4Address :461-468)
    if (windows(fam) && arch == "amd64")
        cap[R_PRIVIP] = in.has_vpc_limits ? ((int64_t)in.vpc_ipv4_per_interface - 1) * 1000 : 0;

    // ---- Overhead (types.go:140-146) ----
    int64_t kube[KP_CATALOG_R] = {}, sys[KP_CATALOG_R] = {}, ev[KP_CATALOG_R] = {};
    {  // kubeReservedResources (:493-530)
        const int64_t kpods = f.eni_mem ? eni_limited_pods(in, 0) : pods;
        kube[R_MEM] = (11 * kpods + 255) * 1024 * 1024 * 1000;
        kube[R_EPH] = ((int64_t)1 << 30) * 1000;
        const int64_t cpu = (int64_t)in.default_vcpus * 1000;
        struct Rng {
            int64_t start, end;
            double pct;
        };
        const Rng rs[4] = {{0, 1000, 0.06}, {1000, 2000, 0.01}, {2000, 4000, 0.005}, {4000, (int64_t)1 << 31, 0.0025}};
        int64_t kc = 0;
        for (const Rng& r : rs) {
            if (cpu >= r.start) {
                double x = (double)(r.end - r.start);
                if (cpu < r.end) x = (double)(cpu - r.start);
                kc += (int64_t)(x * r.pct);
            }
        }
        kube[R_CPU] = kc;
        for (int i = 0; i < nc.n_kube_reserved; i++) {  // lo.Assign: user values replace the defaults
            const int r = resource_index(nc.kube_reserved[i].key);
            int64_t m;
            if (!quantity_milli(nc.kube_reserved[i].value, &m)) throw Err{"malformed kubeReserved quantity"};
            if (r >= 0) kube[r] = m;
        }
    }
    for (int i = 0; i < nc.n_system_reserved; i++) {  // systemReservedResources (:487-491)
        const int r = resource_index(nc.system_reserved[i].key);
        int64_t m;
        if (!quantity_milli(nc.system_reserved[i].value, &m)) throw Err{"malformed systemReserved quantity"};
        if (r >= 0) sys[r] = m;
    }
    {  // evictionThreshold (:532-560)
        const int64_t eph_bytes = ceil_div_1000(eph_m);
        ev[R_MEM] = 100LL * 1024 * 1024 * 1000;
        ev[R_EPH] = (int64_t)std::ceil((double)eph_bytes / 100 * 10) * 1000;
        int64_t ov[KP_CATALOG_R] = {};
        bool ov_set[KP_CATALOG_R] = {};
        auto signals = [&](int n, const kp_string_pair* m) {
            int64_t t[KP_CATALOG_R] = {};
            bool ts[KP_CATALOG_R] = {};
            for (int i = 0; i < n; i++) {
                if (!m[i].key || !m[i].value) continue;
                if (!strcmp(m[i].key, "memory.available")) t[R_MEM] = eviction_signal(mem, m[i].value), ts[R_MEM] = true;
                else if (!strcmp(m[i].key, "nodefs.available")) t[R_EPH] = eviction_signal(eph_bytes, m[i].value), ts[R_EPH] = true;
            }
            for (int r = 0; r < KP_CATALOG_R; r++)  // resources.MaxResources
                if (ts[r]) {
                    ov[r] = ov_set[r] ? std::max(ov[r], t[r]) : t[r];
                    ov_set[r] = true;
                }
        };
        if (nc.eviction_hard) signals(nc.n_eviction_hard, nc.eviction_hard);
        if (nc.eviction_soft && f.evsoft) signals(nc.n_eviction_soft, nc.eviction_soft);
        for (int r = 0; r < KP_CATALOG_R; r++)
            if (ov_set[r]) ev[r] = ov[r];
    }
    for (int r = 0; r < KP_CATALOG_R; r++) b.ovh[r] = kube[r] + sys[r] + ev[r];
    return b;
}

}  // namespace

struct kp_catalog {
    std::vector<std::string> keys;
    std::vector<const char*> key_ptrs;
    std::vector<std::string> names;
    std::vector<const char*> name_ptrs;
    std::vector<const char*> res_ptrs;
    std::vector<int64_t> cap, alloc, ovh;
    std::vector<int8_t> state;
    std::vector<int32_t> offsets;
    std::vector<std::string> values;
    std::vector<const char*> value_ptrs;
    std::vector<int32_t> o_type, o_cap;
    std::vector<double> o_price;
    std::vector<uint8_t> o_avail;
    std::vector<int8_t> o_state;
    std::vector<std::string> o_vals;
    std::vector<const char*> o_val_ptrs, o_key_ptrs;
};

extern "C" kp_status kp_catalog_build(int32_t n_types, const kp_ec2_instance_type* types, const kp_nodeclass_view* nc,
                                      const kp_offering_source* os, kp_catalog** out) {
    if (!out || n_types < 0 || (n_types > 0 && !types) || !nc || !os) return KP_E_INVALID;
    *out = nullptr;
    if (nc->ami_family < KP_AMI_AL2 || nc->ami_family > KP_AMI_CUSTOM) return KP_E_INVALID;
    if (os->n_zones < 0 || (os->n_zones > 0 && !os->zones) || (n_types > 0 && (!os->type_zones || !os->od_price)))
        return KP_E_INVALID;
    auto bad_array = [](int32_t n, const void* p) { return n < 0 || (n > 0 && !p); };
    if (bad_array(nc->n_zones, nc->zones) || bad_array(nc->n_block_device_mappings, nc->block_device_mappings) ||
        bad_array(nc->n_kube_reserved, nc->kube_reserved) || bad_array(nc->n_system_reserved, nc->system_reserved) ||
        (nc->eviction_hard && nc->n_eviction_hard < 0) || (nc->eviction_soft && nc->n_eviction_soft < 0) ||
        bad_array(nc->n_capacity_reservations, nc->capacity_reservations))
        return KP_E_INVALID;
    try {
        auto owned = std::make_unique<kp_catalog>();  // freed if building any type throws
        kp_catalog* c = owned.get();
        const int Z = os->n_zones;
        std::map<std::string, std::string> zone_id;  // subnetZonesToZoneIDs (offering.go:75-77): the last subnet wins
        for (int i = 0; i < nc->n_zones; i++)
            if (nc->zones[i].zone) zone_id[nc->zones[i].zone] = nc->zones[i].zone_id ? nc->zones[i].zone_id : "";
        c->keys = type_keys();
        const int K = (int)c->keys.size();
        for (int r = 0; r < KP_CATALOG_R; r++) c->res_ptrs.push_back(kResources[r]);
        std::vector<std::vector<std::string>> vals_tk;
        for (int t = 0; t < n_types; t++) {
            const kp_ec2_instance_type& in = types[t];
            if (in.n_network_cards > 0 && (!in.card_max_interfaces || in.default_card < 0 || in.default_card >= in.n_network_cards))
                throw Err{"network card index out of range"};
            if ((in.n_gpus > 0 && !in.gpus) || (in.n_accelerators > 0 && !in.accelerators) || (in.n_neuron > 0 && !in.neuron) ||
                (in.n_architectures > 0 && !in.architectures) || (in.n_usage_classes > 0 && !in.usage_classes))
                throw Err{"missing array"};
            std::vector<std::string> offz;
            if (os->type_zones[t]) {
                const std::string s = os->type_zones[t];
                size_t st = 0;
                while (st <= s.size()) {
                    const size_t d = s.find('\n', st);
                    const std::string z = s.substr(st, d == std::string::npos ? std::string::npos : d - st);
                    if (!z.empty()) offz.push_back(z);
                    if (d == std::string::npos) break;
                    st = d + 1;
                }
            }
            Built b = build_type(in, *nc, offz);
            c->names.push_back(b.name);
            for (int r = 0; r < KP_CATALOG_R; r++) {
                c->cap.push_back(b.cap[r]);
                c->ovh.push_back(b.ovh[r]);
                c->alloc.push_back(b.cap[r] - b.ovh[r]);  // resources.Subtract(Capacity, Overhead.Total())
            }
            for (int k = 0; k < K; k++) {
                const std::string& key = c->keys[k];
                c->offsets.push_back((int32_t)c->values.size());
                if (b.absent.count(key)) {
                    c->state.push_back(KP_LABEL_ABSENT);
                    continue;
                }
                const auto& v = b.labels[key];
                c->state.push_back(v.empty() ? KP_LABEL_DOES_NOT_EXIST : KP_LABEL_IN);
                for (const auto& x : v) c->values.push_back(x);
            }
            // ---- createOfferings (offering.go:103-196) ----
            const std::vector<std::string>& itz = b.labels[K_ZONE];
            const std::set<std::string> it_zones(itz.begin(), itz.end());
            auto offer = [&](const char* ct, const std::string& zone, double price, bool available, int32_t rcap,
                             const char* rid, const char* rtype) {
                c->o_type.push_back(t);
                c->o_price.push_back(price);
                c->o_avail.push_back(available ? 1 : 0);
                c->o_cap.push_back(rcap);
                const auto zi = zone_id.find(zone);
                const char* v[5] = {ct, zone.c_str(), rid, rtype, zi != zone_id.end() ? zi->second.c_str() : nullptr};
                for (int q = 0; q < 5; q++) {
                    if (q == 4) c->o_state.push_back(v[q] ? KP_LABEL_IN : KP_LABEL_ABSENT);
                    else c->o_state.push_back(v[q] ? KP_LABEL_IN : KP_LABEL_DOES_NOT_EXIST);
                    c->o_vals.push_back(v[q] ? v[q] : "");
                }
            };
            const double od = os->od_price[t];
            const bool has_od = !std::isnan(od);
            for (int zi = 0; zi < Z; zi++) {
                const std::string zone = os->zones[zi] ? os->zones[zi] : "";
                for (const auto& ct : b.labels[K_CT]) {
                    if (ct == "reserved") continue;
                    const int cti = ct == "on-demand" ? 0 : 1;
                    const bool ice = os->unavailable && os->unavailable[((size_t)t * Z + zi) * 2 + cti];
                    double price = 0.0;
                    bool has = false;
                    if (cti == 0) {
                        has = has_od;
                        price = has ? od : 0.0;
                    } else {
                        const double sp = os->spot_price ? os->spot_price[(size_t)t * Z + zi] : NAN;
                        has = !std::isnan(sp);
                        price = has ? sp : 0.0;
                    }
                    offer(ct.c_str(), zone, price, !ice && has && it_zones.count(zone), 0, nullptr, nullptr);
                }
            }
            if (nc->reserved_capacity) {
                for (int i = 0; i < nc->n_capacity_reservations; i++) {
                    const kp_capacity_reservation& cr = nc->capacity_reservations[i];
                    if (!cr.instance_type || strcmp(cr.instance_type, in.name)) continue;
                    const std::string zone = cr.availability_zone ? cr.availability_zone : "";
                    const double price = has_od ? od / 10000000.0 : 0.0;
                    offer("reserved", zone, price,
                          cr.available_count != 0 && it_zones.count(zone) && !cr.expiring, cr.available_count,
                          cr.id ? cr.id : "", cr.reservation_type ? cr.reservation_type : "");
                }
            }
        }
        c->offsets.push_back((int32_t)c->values.size());
        for (const auto& k : c->keys) c->key_ptrs.push_back(k.c_str());
        for (const auto& n : c->names) c->name_ptrs.push_back(n.c_str());
        for (const auto& v : c->values) c->value_ptrs.push_back(v.c_str());
        for (const auto& v : c->o_vals) c->o_val_ptrs.push_back(v.c_str());
        for (int q = 0; q < 5; q++) c->o_key_ptrs.push_back(kOfferingKeys[q]);
        *out = owned.release();
        return KP_OK;
    } catch (const Err&) {
        return KP_E_INVALID;
    } catch (...) {
        return KP_E_INVALID;
    }
}

extern "C" kp_status kp_catalog_get_view(const kp_catalog* c, kp_catalog_view* v) {
    if (!c || !v) return KP_E_INVALID;
    memset(v, 0, sizeof(*v));
    v->n_types = (int32_t)c->names.size();
    v->n_resources = KP_CATALOG_R;
    v->resource_names = c->res_ptrs.data();
    v->type_names = c->name_ptrs.data();
    v->capacity = c->cap.data();
    v->allocatable = c->alloc.data();
    v->n_label_keys = (int32_t)c->keys.size();
    v->label_keys = c->key_ptrs.data();
    v->label_state = c->state.data();
    v->label_offsets = c->offsets.data();
    v->label_values = c->value_ptrs.data();
    v->n_offerings = (int32_t)c->o_type.size();
    v->offering_type = c->o_type.data();
    v->offering_price = c->o_price.data();
    v->offering_available = c->o_avail.data();
    v->offering_reservation_capacity = c->o_cap.data();
    v->n_offering_keys = 5;
    v->offering_keys = c->o_key_ptrs.data();
    v->offering_label_state = c->o_state.data();
    v->offering_label_values = c->o_val_ptrs.data();
    return KP_OK;
}

extern "C" kp_status kp_catalog_overhead(const kp_catalog* c, int32_t t, int64_t* overhead) {
    if (!c || !overhead || t < 0 || t >= (int32_t)c->names.size()) return KP_E_INVALID;
    memcpy(overhead, c->ovh.data() + (size_t)t * KP_CATALOG_R, sizeof(int64_t) * KP_CATALOG_R);
    return KP_OK;
}

extern "C" const char* kp_catalog_resource_name(int32_t r) {
    return r >= 0 && r < KP_CATALOG_R ? kResources[r] : nullptr;
}

extern "C" kp_status kp_catalog_free(kp_catalog* c) {
    delete c;
    return KP_OK;
}
