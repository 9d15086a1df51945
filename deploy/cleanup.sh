#!/usr/bin/env bash
# Remove the training job (and with --all the Aim server and both volumes: deletes checkpoints and runs).
set -uo pipefail
kubectl delete job "${JOB:-smollm3-sft-mi355x}" --ignore-not-found
if [ "${1:-}" = "--all" ]; then
  kubectl delete -f deploy/aim/aim.yaml --ignore-not-found
  kubectl delete -f deploy/storage.yaml --ignore-not-found
fi
