# Multi-process rehearsal on one GPU (EDGE_SHARED_GPU=1: gloo group, host-staged p2p, every rank on cuda:0).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
B="bench.py --steps 3 --warmup 1"
timeout -k 10 300 python $B > gpurun_out/reh_n1.log 2>&1; rc=$?; echo "[n1] rc=$rc $(grep -o '"value": [0-9.]*\|"ppl_random_weights": [0-9.]*' gpurun_out/reh_n1.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
export EDGE_SHARED_GPU=1
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 300 $TR --nproc-per-node 2 --master-port 29611 $B --gpus 2 > gpurun_out/reh_n2.log 2>&1; rc=$?; echo "[n2] rc=$rc $(grep -o '"value": [0-9.]*\|"ppl_random_weights": [0-9.]*\|"parallelism": "[a-z0-9]*"' gpurun_out/reh_n2.log | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -30 gpurun_out/reh_n2.log; exit $rc; }
EDGE_P2P_CHECK=1 timeout -k 10 300 $TR --nproc-per-node 2 --master-port 29612 $B --gpus 2 --no-graphs > gpurun_out/reh_n2c.log 2>&1; rc=$?; echo "[n2 checked, eager] rc=$rc $(grep -o '"ppl_random_weights": [0-9.]*' gpurun_out/reh_n2c.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/reh_n2c.log; exit $rc; }
timeout -k 10 300 $TR --nproc-per-node 4 --master-port 29613 $B --gpus 4 > gpurun_out/reh_n4.log 2>&1; rc=$?; echo "[n4] rc=$rc $(grep -o '"ppl_random_weights": [0-9.]*\|"parallelism": "[a-z0-9]*"' gpurun_out/reh_n4.log | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -30 gpurun_out/reh_n4.log; exit $rc; }
cd Experiments/Pipeline
timeout -k 10 300 python main.py --params configs/config4_qwen2_4stage_lastrow.json --max-windows 48 --dataset synthetic > ../../gpurun_out/reh_pipe1.log 2>&1; rc=$?; echo "[pipe local] rc=$rc"; grep "ratio=" ../../gpurun_out/reh_pipe1.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $TR --nproc-per-node 4 --master-port 29614 main.py --params configs/config4_qwen2_4stage_lastrow.json --max-windows 48 --dataset synthetic > ../../gpurun_out/reh_pipe4.log 2>&1; rc=$?; echo "[pipe 4 ranks] rc=$rc"; grep "ratio=" ../../gpurun_out/reh_pipe4.log | cut -c1-150; [ $rc -eq 0 ] || { tail -30 ../../gpurun_out/reh_pipe4.log; exit $rc; }
