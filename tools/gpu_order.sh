# VGPR-bank / slow-fast sequence probe, then the SHA-256 round-order search.
set -u
mkdir -p gpurun_out
timeout -k 10 120 ./tools/bank_probe > gpurun_out/bank_probe2.json
rc=$?; echo "bank rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 ./tools/order_search > gpurun_out/order_search.json
rc=$?; echo "order rc=$rc"; cat gpurun_out/order_search.json; exit $rc
