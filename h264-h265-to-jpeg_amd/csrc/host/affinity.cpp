// Host-thread placement: see affinity.h.  Sysfs paths are read under $H2J_SYSFS_ROOT (default
// "/sys") so the CPU tests can run the plan against a fake topology.
#include "affinity.h"

#include <sched.h>

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace h2j {

namespace {

std::string sysfs(const std::string& rel) {
    const char* r = std::getenv("H2J_SYSFS_ROOT");
    return std::string(r && *r ? r : "/sys") + rel;
}

bool read_line(const std::string& path, std::string& out) {
    std::ifstream f(path);
    if (!f) return false;
    std::getline(f, out);
    return true;
}

}  // namespace

std::vector<int> parse_cpulist(const std::string& s) {
    std::vector<int> out;
    std::stringstream ss(s);
    std::string part;
    while (std::getline(ss, part, ',')) {
        while (!part.empty() && std::isspace(static_cast<unsigned char>(part.back()))) part.pop_back();
        while (!part.empty() && std::isspace(static_cast<unsigned char>(part.front()))) part.erase(part.begin());
        if (part.empty()) continue;
        const size_t dash = part.find('-');
        char* end = nullptr;
        const long a = std::strtol(part.c_str(), &end, 10);
        long b = a;
        if (dash != std::string::npos) b = std::strtol(part.c_str() + dash + 1, &end, 10);
        if (a < 0 || b < a || b - a > 65536) continue;
        for (long c = a; c <= b; c++) out.push_back(static_cast<int>(c));
    }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out;
}

std::vector<int> process_cpus() {
    std::vector<int> out;
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof(set), &set) == 0)
        for (int c = 0; c < CPU_SETSIZE; c++)
            if (CPU_ISSET(c, &set)) out.push_back(c);
    return out;
}

double cgroup_cpu_quota() {
    std::string line;
    if (read_line(sysfs("/fs/cgroup/cpu.max"), line)) {  // v2: "<quota> <period>" or "max <period>"
        char q[32] = {0};
        long period = 0;
        if (std::sscanf(line.c_str(), "%31s %ld", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0)
            return std::atof(q) / static_cast<double>(period);
        return 0.0;
    }
    std::string qs, ps;  // v1
    if (read_line(sysfs("/fs/cgroup/cpu/cpu.cfs_quota_us"), qs) && read_line(sysfs("/fs/cgroup/cpu/cpu.cfs_period_us"), ps)) {
        const double q = std::atof(qs.c_str()), p = std::atof(ps.c_str());
        if (q > 0 && p > 0) return q / p;
    }
    return 0.0;
}

int pci_numa_node(const std::string& bus_id) {
    std::string id = bus_id;
    for (char& c : id) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    std::string line;
    if (!read_line(sysfs("/bus/pci/devices/" + id + "/numa_node"), line)) return -1;
    return std::atoi(line.c_str());
}

std::vector<int> node_cpus(int node) {
    std::string line;
    if (node < 0 || !read_line(sysfs("/devices/system/node/node" + std::to_string(node) + "/cpulist"), line)) return {};
    return parse_cpulist(line);
}

int local_procs() {
    for (const char* name : {"H2J_LOCAL_PROCS", "LOCAL_WORLD_SIZE"}) {
        const char* v = std::getenv(name);
        if (v && std::atoi(v) > 0) return std::atoi(v);
    }
    return 1;
}

HostPlan plan_host(int device, const std::vector<int>& device_nodes, const std::vector<int>& cpus,
                   const std::vector<int>& node_cpu_list, double quota, int requested, int engines) {
    HostPlan plan;
    engines = std::max(1, engines);
    const int node = device >= 0 && device < static_cast<int>(device_nodes.size()) ? device_nodes[device] : -1;
    plan.numa_node = node;
    // candidate CPUs: the process mask on the device's node (the whole mask if the node is
    // unknown or the mask has none of its CPUs)
    std::vector<int> cand;
    for (int c : cpus)
        if (std::binary_search(node_cpu_list.begin(), node_cpu_list.end(), c)) cand.push_back(c);
    int rank = 0, mates = 1;
    if (cand.empty()) {
        cand = cpus;
        // unknown topology: split the mask between all visible devices
        rank = device;
        mates = std::max(1, static_cast<int>(device_nodes.size()));
    } else {
        mates = 0;
        for (size_t i = 0; i < device_nodes.size(); i++) {
            if (device_nodes[i] != node) continue;
            if (static_cast<int>(i) < device) rank++;
            mates++;
        }
        mates = std::max(1, mates);
    }
    std::vector<int> slice;
    const size_t n = cand.size();
    if (n >= static_cast<size_t>(mates)) {
        const size_t a = n * static_cast<size_t>(rank) / static_cast<size_t>(mates);
        const size_t b = n * static_cast<size_t>(rank + 1) / static_cast<size_t>(mates);
        slice.assign(cand.begin() + static_cast<long>(a), cand.begin() + static_cast<long>(b));
    } else {
        slice = cand;  // fewer CPUs than devices: share them
    }
    int t = requested;
    if (t <= 0) {
        t = static_cast<int>(slice.size());
        // the cgroup quota is shared by every engine of every process of the node's job
        if (quota > 0) t = std::min(t, std::max(1, static_cast<int>(std::ceil(quota / (engines * local_procs())))));
        t = std::min(t, 64);
    }
    plan.threads = std::max(1, t);
    const char* pin = std::getenv("H2J_PIN");
    if (!(pin && std::strcmp(pin, "0") == 0)) plan.cpus = slice;
    return plan;
}

}  // namespace h2j
