mkdir -p gpurun_out
for r in 10000000 1250000; do
  VS_ABL_SET=qmax VS_ABL_BURST=8 timeout -k 10 200 ./tools/ablate_mfma $r 16 > gpurun_out/r04_abl_qmax_ab_$r.txt 2>&1 || exit 1
  head -10 gpurun_out/r04_abl_qmax_ab_$r.txt
done
for st in 5 7 9 12; do
  VS_ABL_SET=product VS_ABL_BURST=8 timeout -k 10 200 ./tools/ablate_mfma 10000000 10 $st > gpurun_out/r04_abl_st_10m_$st.txt 2>&1 || exit 1
  echo "st=$st"; head -10 gpurun_out/r04_abl_st_10m_$st.txt | grep -E "sample|main|qmax full|slabs"
done
for st in 2 3 4 6; do
  VS_ABL_SET=product VS_ABL_BURST=8 timeout -k 10 200 ./tools/ablate_mfma 1250000 10 $st > gpurun_out/r04_abl_st_1p25m_$st.txt 2>&1 || exit 1
  echo "st=$st"; head -10 gpurun_out/r04_abl_st_1p25m_$st.txt | grep -E "sample|main|qmax full|slabs"
done
