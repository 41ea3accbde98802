set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 120 ./tools/ubench_field > $O/ubench_field.jsonl
timeout -k 10 60 ./tools/ubench_valu > $O/ubench_valu.json
echo ALLDONE
