# Round-4 final bench line (after tools/r04_final.sh's profiles were summarised here and the PMC
# summary stamped with the loaded unit), then smoke().
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
