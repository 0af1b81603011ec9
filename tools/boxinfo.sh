# Host facts of the GPU box that bear on the host half of ValidateBatch
# (VERDICT r04 item 1): NUMA layout, automatic NUMA balancing, THP, the cgroup's
# CPU quota / memory limits, malloc-relevant limits.  CPU only.
echo "== lscpu"; lscpu | grep -Ei "model name|socket|numa|^cpu\(s\)|thread"
echo "== numa_balancing"; cat /proc/sys/kernel/numa_balancing 2>&1
echo "== thp enabled / defrag"; cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag 2>&1
echo "== cgroup"; for f in cpu.max cpu.stat memory.max memory.current memory.high cpuset.cpus.effective cpuset.mems.effective; do printf "%s: " $f; tr '\n' ' ' < /sys/fs/cgroup/$f 2>&1; echo; done
echo "== affinity"; python3 -c "import os; a=sorted(os.sched_getaffinity(0)); print(len(a), a[:4], a[-4:])"
echo "== numa nodes"; for n in /sys/devices/system/node/node*; do echo "$n $(cat $n/cpulist) $(grep MemTotal $n/meminfo)"; done 2>&1 | head -16
echo "== gpu numa"; cat /sys/class/drm/card*/device/numa_node 2>/dev/null | tr '\n' ' '; echo
echo "== glibc"; ldd --version | head -1
