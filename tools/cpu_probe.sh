#!/usr/bin/env bash
# Host CPU facts of the GPU box (tools only): cgroup quota, affinity, topology, load.
echo "nproc: $(nproc)"
echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
echo "cpuset.cpus.effective: $(cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null)"
echo "loadavg: $(cat /proc/loadavg)"
lscpu | grep -E "Model name|Socket|Core|Thread|NUMA" || true
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
