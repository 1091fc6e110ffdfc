# Render every sample scene through the C++ CLI (PNG + PFM) into gpurun_out/scenes/.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/scenes
python -c "import __graft_entry__ as g; g.build_host()" || exit 1
for s in box square_lit_by_square lit_corner fractal smallpt spheres:2000 box_lights:16; do
  n=${s%%:*}
  timeout -k 10 120 ./ipt_amd/bin/ipt_render --scene $s --width 320 --height 320 --spp 64 --passes 2 \
    --out gpurun_out/scenes/$n.png --pfm gpurun_out/scenes/$n.pfm > gpurun_out/scenes/$n.json || { echo "$s failed"; exit 1; }
  cat gpurun_out/scenes/$n.json
done
