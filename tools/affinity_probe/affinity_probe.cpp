// CPU test driver for csrc/host/affinity.cpp (tests/test_affinity.py):
//   affinity_probe plan <device> <node,node,...> <process cpulist> <quota> <requested> <engines>
//     -> "threads=<t> node=<n> cpus=<cpulist>" using the node cpulists under $H2J_SYSFS_ROOT
//   affinity_probe sysfs <pci bus id>
//     -> "numa=<n> quota=<q>" read from $H2J_SYSFS_ROOT
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <string>
#include <vector>

#include "affinity.h"

int main(int argc, char** argv) {
    if (argc >= 8 && !std::strcmp(argv[1], "plan")) {
        const int dev = std::atoi(argv[2]);
        std::vector<int> nodes;
        std::stringstream ss(argv[3]);
        std::string t;
        while (std::getline(ss, t, ',')) nodes.push_back(std::atoi(t.c_str()));
        const int node = dev < static_cast<int>(nodes.size()) ? nodes[dev] : -1;
        h2j::HostPlan p = h2j::plan_host(dev, nodes, h2j::parse_cpulist(argv[4]), h2j::node_cpus(node),
                                         std::atof(argv[5]), std::atoi(argv[6]), std::atoi(argv[7]));
        std::printf("threads=%d node=%d cpus=", p.threads, p.numa_node);
        for (size_t i = 0; i < p.cpus.size(); i++) std::printf(i ? ",%d" : "%d", p.cpus[i]);
        std::printf("\n");
        return 0;
    }
    if (argc >= 3 && !std::strcmp(argv[1], "sysfs")) {
        std::printf("numa=%d quota=%g\n", h2j::pci_numa_node(argv[2]), h2j::cgroup_cpu_quota());
        return 0;
    }
    std::fprintf(stderr, "usage: affinity_probe plan|sysfs ...\n");
    return 2;
}
