bash tools/gpu/r04h.sh && bash tools/gpu/r04i.sh
