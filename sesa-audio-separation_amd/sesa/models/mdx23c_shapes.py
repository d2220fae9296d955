"""Parameter names/shapes of TFC_TDF_net in the reference named_parameters() order
(models/mdx23c_tfc_tdf_v3.py:100-189).  Mirrors the native registry in csrc/sesa_mdx23c.hip."""


def param_shapes(c):
    """c: dict with the keys of sesa_mdx23c_config (chunk_size, dim_f, num_subbands, ...)."""
    k = c["num_subbands"]
    dim_c = k * c["audio_channels"] * 2
    n, l, ch, g, bn = c["num_scales"], c["num_blocks_per_scale"], c["num_channels"], c["growth"], c["bottleneck_factor"]
    st, sf = c["scale_t"], c["scale_f"]
    f = c["dim_f"] // k
    out = [("first_conv.weight", (ch, dim_c, 1, 1))]

    def stack(prefix, in_c, c_, f_):
        for i in range(l):
            p = f"{prefix}.blocks.{i}"
            out.extend([
                (f"{p}.tfc1.0.weight", (in_c,)), (f"{p}.tfc1.0.bias", (in_c,)), (f"{p}.tfc1.2.weight", (c_, in_c, 3, 3)),
                (f"{p}.tdf.0.weight", (c_,)), (f"{p}.tdf.0.bias", (c_,)), (f"{p}.tdf.2.weight", (f_ // bn, f_)),
                (f"{p}.tdf.3.weight", (c_,)), (f"{p}.tdf.3.bias", (c_,)), (f"{p}.tdf.5.weight", (f_, f_ // bn)),
                (f"{p}.tfc2.0.weight", (c_,)), (f"{p}.tfc2.0.bias", (c_,)), (f"{p}.tfc2.2.weight", (c_, c_, 3, 3)),
                (f"{p}.shortcut.weight", (c_, in_c, 1, 1))])
            in_c = c_

    for i in range(n):
        stack(f"encoder_blocks.{i}.tfc_tdf", ch, ch, f)
        out += [(f"encoder_blocks.{i}.downscale.conv.0.weight", (ch,)),
                (f"encoder_blocks.{i}.downscale.conv.0.bias", (ch,)),
                (f"encoder_blocks.{i}.downscale.conv.2.weight", (ch + g, ch, st, sf))]
        f //= sf
        ch += g
    stack("bottleneck_block", ch, ch, f)
    for i in range(n):
        out += [(f"decoder_blocks.{i}.upscale.conv.0.weight", (ch,)),
                (f"decoder_blocks.{i}.upscale.conv.0.bias", (ch,)),
                (f"decoder_blocks.{i}.upscale.conv.2.weight", (ch, ch - g, st, sf))]
        f *= sf
        ch -= g
        stack(f"decoder_blocks.{i}.tfc_tdf", 2 * ch, ch, f)
    out.append(("final_conv.0.weight", (ch, ch + dim_c, 1, 1)))
    out.append(("final_conv.2.weight", (c["num_instruments"] * dim_c, ch, 1, 1)))
    return out
