#!/usr/bin/env bash
# Start a master and N check slaves (reference: bin/comm_cluster_error_check.sh).
# Local by default; set SLAVE_HOSTS="h1 h2 ..." and LOGIN_USER to fan out over ssh.
#   SLAVE_NUM=4 MODE=process bin/mp4x_check.sh
set -u
cd "$(dirname "$0")/.."
SLAVE_NUM=${SLAVE_NUM:-4}
THREAD_NUM=${THREAD_NUM:-2}
MASTER_HOST=${MASTER_HOST:-127.0.0.1}
MASTER_PORT=${MASTER_PORT:-61235}
ARR_SIZE=${ARR_SIZE:-1000000}
OBJ_SIZE=${OBJ_SIZE:-1000}
RUN_TIME=${RUN_TIME:-3}
MODE=${MODE:-process}
export MP4X_LOG_DIR=${MP4X_LOG_DIR:-log}
COMPRESS=${COMPRESS:-false}
TEST_RPC=${TEST_RPC:-false}
DEVICE=${DEVICE:-cpu}
LOGIN_USER=${LOGIN_USER:-$USER}
SLAVE_HOSTS=${SLAVE_HOSTS:-}
mkdir -p log
[ -f "kill_${MASTER_PORT}.sh" ] && sh "kill_${MASTER_PORT}.sh" 2>/dev/null
python -m mp4x.control.master "$SLAVE_NUM" "$MASTER_PORT" > log/master.log 2>&1 &
MASTER_PID=$!
echo $MASTER_PID > "master_${MASTER_PORT}.pid"
CMD="python -m mp4x.check $LOGIN_USER $MASTER_HOST $MASTER_PORT $ARR_SIZE $OBJ_SIZE $RUN_TIME $THREAD_NUM $MODE $COMPRESS $TEST_RPC --device $DEVICE"
if [ -z "$SLAVE_HOSTS" ]; then
  for i in $(seq 1 "$SLAVE_NUM"); do $CMD > "log/slave_$i.log" 2>&1 & done
else
  for h in $SLAVE_HOSTS; do ssh "$LOGIN_USER@$h" "cd $(pwd) && nohup $CMD > log/slave.log 2>&1 &"; done
fi
wait $MASTER_PID
CODE=$?
echo "master exit code: $CODE"
exit $CODE
