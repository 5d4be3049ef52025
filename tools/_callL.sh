bash tools/gpu.sh suite r03/final3 && bash tools/gpu.sh bench r03/final3b --steps 20 --warmup 5
