QDML_DBG=1 QDML_DIST_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 tests/dist_scripts/flagship_dp.py gpurun_out/fl cuda > gpurun_out/dbg_fl.log 2>&1
cat gpurun_out/fl.0 gpurun_out/fl.1 >> gpurun_out/dbg_fl.log
