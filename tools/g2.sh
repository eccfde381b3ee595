cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/g2
cat /sys/fs/cgroup/cpu.max > gpurun_out/g2/cgroup.txt 2>&1; nproc --all >> gpurun_out/g2/cgroup.txt
timeout -k 10 900 python bench.py > gpurun_out/g2/bench.json 2> gpurun_out/g2/bench.err
