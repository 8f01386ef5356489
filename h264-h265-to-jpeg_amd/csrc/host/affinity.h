// Host-thread placement for the entropy pools ("each GPU gets its own host
// entropy thread pool, NUMA-local").  The engine on device d runs its pool on the CPUs of the
// process affinity mask that sit on d's NUMA node, split evenly between the visible devices of
// that node (d takes the slice of its rank among them), so N engines in one process, or N
// single-GPU processes under torchrun, get disjoint NUMA-local CPU sets without the launcher
// slicing affinity itself.  Thread count: the slice size, bounded by the cgroup CPU quota
// (divided between the engines of the process) and 64.
#pragma once
#include <string>
#include <vector>

namespace h2j {

struct HostPlan {
    std::vector<int> cpus;  // CPUs the pool's workers are pinned to (empty: not pinned)
    int threads = 1;        // pool size including the calling thread
    int numa_node = -1;     // the device's NUMA node (-1 unknown)
};

std::vector<int> parse_cpulist(const std::string& s);  // "0-3,8,10-11" -> {0,1,2,3,8,10,11}
std::vector<int> process_cpus();                      // sched_getaffinity
double cgroup_cpu_quota();                             // cores (cgroup v2 cpu.max / v1 cfs), 0 = none
int pci_numa_node(const std::string& bus_id);          // sysfs numa_node of a PCI device, -1 unknown
std::vector<int> node_cpus(int node);                  // sysfs cpulist of a NUMA node

// processes of this job on the node that share the cgroup CPU quota: $H2J_LOCAL_PROCS, else
// torchrun's $LOCAL_WORLD_SIZE, else 1
int local_procs();

// device_nodes[i]: NUMA node of visible device i.  requested > 0 fixes the thread count;
// engines: engines of this process; the cgroup quota is divided by engines x local_procs().
// H2J_PIN=0 disables pinning.
HostPlan plan_host(int device, const std::vector<int>& device_nodes, const std::vector<int>& cpus,
                   const std::vector<int>& node_cpu_list, double quota, int requested, int engines);

}  // namespace h2j
