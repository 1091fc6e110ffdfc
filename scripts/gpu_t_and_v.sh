# GPU parity tests, then C2 A/B of library variants ($VARIANTS) and, with
# $OCC set, C2 throughput at fewer resident workgroups per CU
bash scripts/gpu_tests.sh && VARIANTS="${VARIANTS}" bash scripts/gpu_variants.sh && { [ -z "$OCC" ] || bash scripts/gpu_occupancy.sh; }
