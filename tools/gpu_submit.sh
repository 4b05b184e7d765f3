#!/bin/bash
# Host side (this container): submit one gpurun command, re-submitting only while the pod has
# no free GPU slot (gpurun exit 3: nothing ran, nothing charged), at most N tries, 4 min apart.
# Any other outcome -- success, a failing command, a refusal -- ends it.  Log in LOG.
# usage: bash tools/gpu_submit.sh LOG TIMEOUT_S CMD...
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
    /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
    rc=$?
    echo "[submit] try $i rc=$rc" >> "$LOG"
    if [ $rc -ne 3 ] && ! grep -q "GPU slot(s) on this pod are busy\|box was taken away" "$LOG"; then break; fi
    sleep 240
done
echo done >> "$LOG"
