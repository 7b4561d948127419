#!/bin/bash
# Training ranks only (reference scripts/run_dist_tf_daint.sh): same environment interface as
# run_dist_train_eval.sh without the eval sidecar.
unset TF_EVAL_SCRIPT
exec "$(dirname "${BASH_SOURCE[0]}")/run_dist_train_eval.sh" "$@"
