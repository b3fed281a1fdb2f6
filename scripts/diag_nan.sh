cd $GRAFT_REPO_ROOT; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/diag_nan3.log; : > $O
SHORT=1 PDT_NAN_TRACE=1 FILL_NAN=1 timeout -k 10 200 python scripts/diag_race.py >> $O 2>&1 || exit 1
