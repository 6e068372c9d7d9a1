cd $GRAFT_REPO_ROOT && timeout -k 10 200 python tools/diag_fix.py 2>&1 | tail -2
