set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
export MIOPEN_FIND_MODE=FAST
P="python3 scripts/probes/probe_roofline.py"
F="pgemm|syrk|tile_reduce|factor_ema|gather_grad|split_copy"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && \
bash scripts/prof_run.sh roof_kt 300 -- $P && \
bash scripts/pmc_run.sh roof_m 300 "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_LDS" --filter "$F" -- $P && \
bash scripts/pmc_run.sh roof_f 300 "FETCH_SIZE" --filter "$F" -- $P && \
bash scripts/pmc_run.sh roof_w 300 "WRITE_SIZE" --filter "$F" -- $P
echo rc=$?
