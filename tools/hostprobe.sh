#!/bin/bash
# Host facts of a GPU box (CPU baseline sizing): CPUs, affinity, cgroup quota, NUMA.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
{
  echo "nproc: $(nproc)"
  python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"
  echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
  grep -i cpus_allowed_list /proc/self/status
  for n in /sys/devices/system/node/node*/cpulist; do echo "$n: $(cat "$n")"; done
  lscpu | head -30
  free -g
} > gpurun_out/hostprobe.txt 2>&1
cat gpurun_out/hostprobe.txt
