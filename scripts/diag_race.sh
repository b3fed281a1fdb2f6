cd $GRAFT_REPO_ROOT; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/diag_race6.log; : > $O
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "sink or captured or mirror or handoff" >> $O 2>&1; echo "pytest rc=$?" >> $O
echo "== FILL_NAN" >> $O; FILL_NAN=1 timeout -k 10 200 python scripts/diag_race.py >> $O 2>&1 || exit 1
echo "== plain" >> $O; timeout -k 10 200 python scripts/diag_race.py >> $O 2>&1 || exit 1
