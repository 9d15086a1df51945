#!/usr/bin/env bash
# Job status, pod events, GPU placement and the trainer's last log lines (the reference's monitor script, for
# the one-pod-per-node MI355X job). Inside the pod, `python -m llm_fine_tune_distributed_amd.cli.status`
# prints the run's own view (last step, throughput, checkpoints).
set -uo pipefail
JOB=${JOB:-smollm3-sft-mi355x}
kubectl get job "$JOB" -o wide
POD=$(kubectl get pods -l job-name="$JOB" -o jsonpath='{.items[0].metadata.name}' 2>/dev/null || true)
[ -z "$POD" ] && { echo "no pod yet"; exit 0; }
kubectl get pod "$POD" -o wide
kubectl get events --field-selector involvedObject.name="$POD" --sort-by=.lastTimestamp | tail -n 10
kubectl exec "$POD" -- sh -c 'rocm-smi --showuse --showmemuse --showpower 2>/dev/null | head -n 30' || true
kubectl exec "$POD" -- python -m llm_fine_tune_distributed_amd.cli.status /persistent/models || true
kubectl logs "$POD" --tail="${TAIL:-40}"
