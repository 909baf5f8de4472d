#!/bin/bash
# Host storage probe on the GPU box: what a durable event store can sustain there.
#   bash scripts/gpu_probe_disk.sh <name>     (results under gpurun_out/<name>)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-disk}"
mkdir -p "$O"
{
  echo "== df"; df -hT "$R" /tmp /dev/shm 2>&1
  echo "== mounts"; grep -E " / | /tmp | /root |$(df --output=target "$R" | tail -1) " /proc/mounts 2>&1
  echo "== lsblk"; lsblk -o NAME,SIZE,ROTA,TYPE,MOUNTPOINT 2>&1 | head -40
  echo "== mem"; free -g
  echo "== cpus"; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null
} > "$O/host.txt" 2>&1
python3 -u "$R/scripts/probe_disk.py" "$R/gpurun_out/_probe_disk.dat" > "$O/disk_repo.txt" 2>&1
python3 -u "$R/scripts/probe_disk.py" /tmp/_probe_disk.dat > "$O/disk_tmp.txt" 2>&1
rm -f "$R/gpurun_out/_probe_disk.dat" /tmp/_probe_disk.dat
cat "$O/host.txt" "$O/disk_repo.txt" "$O/disk_tmp.txt"
