#!/usr/bin/env bash
# Build + push the ROCm image, then submit storage, the Aim server and the 8-GPU MI355X job.
#   REGISTRY=quay.io/me TAG=v0.3 deploy/deploy.sh [--no-build] [--no-aim]
set -euo pipefail
cd "$(dirname "$0")/.."
REGISTRY=${REGISTRY:?set REGISTRY}
TAG=${TAG:-$(python -c 'import llm_fine_tune_distributed_amd as m; print(m.__version__)' 2>/dev/null || echo latest)}
IMAGE="$REGISTRY/llm-fine-tune-distributed-amd:$TAG"
BUILD=1; AIM=1
for a in "$@"; do
  case "$a" in --no-build) BUILD=0 ;; --no-aim) AIM=0 ;; *) echo "unknown option $a" >&2; exit 2 ;; esac
done
if [ "$BUILD" = 1 ]; then
  docker build -f deploy/Dockerfile.rocm -t "$IMAGE" .
  docker push "$IMAGE"
  if [ "$AIM" = 1 ]; then
    docker build -f deploy/aim/Dockerfile -t "$REGISTRY/sftamd-aim:$TAG" deploy/aim
    docker push "$REGISTRY/sftamd-aim:$TAG"
  fi
fi
kubectl apply -f deploy/storage.yaml
if [ "$AIM" = 1 ]; then
  sed "s#REGISTRY/sftamd-aim:latest#$REGISTRY/sftamd-aim:$TAG#" deploy/aim/aim.yaml | kubectl apply -f -
fi
kubectl delete job smollm3-sft-mi355x --ignore-not-found
sed "s#REGISTRY/llm-fine-tune-distributed-amd:latest#$IMAGE#" deploy/job-single-node.yaml | kubectl apply -f -
echo "submitted $IMAGE; follow with deploy/monitor.sh"
