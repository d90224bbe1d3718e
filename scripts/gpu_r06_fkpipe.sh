#!/bin/bash
# r06 fkpipe: FK chunk schedules, same box: alternating streams (default) vs blends in order on one
# stream with each chunk's skinning on the second (TIK_FK_PIPE=1), chunk 2048 / 1024 / 512
cd $GRAFT_REPO_ROOT
O=gpurun_out
TIK_FK_PIPE=1 TIK_FK_CHUNK=1024 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fk.py > $O/pytest_r06fkp.log 2>&1 || { tail -20 $O/pytest_r06fkp.log; exit 1; }
tail -1 $O/pytest_r06fkp.log
for i in 1 2; do
  for v in "0 2048" "1 2048" "1 1024" "1 512"; do
    set -- $v
    TIK_FK_PIPE=$1 TIK_FK_CHUNK=$2 timeout -k 10 120 python -c "
import json, bench_fk; d = bench_fk.measure_fk(4096, 10, 20)
print('pipe $1 chunk $2', d['ms_per_step'], d['value'], ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in d['kernels'].items()))" || exit 1
  done
done | tee $O/ab_r06fkpipe.txt
