#!/bin/bash
# Launch one parameter-server run on a single node: the worker ranks (one
# process per GPU, GPUs 1..N) and the server rank 0 (GPU 0) with CSV logging
# and the reference's producer rate -p 200 (reference run.sh:10-17).  The
# reference's `sleep 10s` ordering hack is unnecessary: both sides meet at the
# torch.distributed rendezvous (127.0.0.1:$MASTER_PORT).  Ctrl-C tears down
# the whole process group (reference run.sh:3-8).
#
# Usage: ./run.sh [NUM_WORKERS] [extra ServerAppRunner flags...]
#   NUM_WORKERS defaults to 4 (the reference's hard-coded numWorkers).
#   Data: ./data/train.csv and ./data/test.csv (see tools/make_data.py).
set -u
cd "$(dirname "$0")"
N="${1:-4}"
shift || true
export MASTER_ADDR=127.0.0.1
export MASTER_PORT="${MASTER_PORT:-29500}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"

trap killgroup SIGINT SIGTERM
killgroup() {
  echo killing...
  kill 0
}

runWorkers() {
  python -m psx.apps.worker_app_runner -l --num_workers "$N"
}

runServer() {
  python -m psx.apps.server_app_runner -l -p 200 --num_workers "$N" "$@"
}

runWorkers & runServer "$@" & wait
