%% raytracer_gpu.erl — the MI355X strategy funs for the reference ray tracer
%% (plouj/eraytracer, raytracer.erl), backed by the rt_nif NIF (erlang/c_src/rt_nif.c)
%% and the HIP library librtmi355x.so.
%%
%% Drop-in for the reference's strategy interface F(Width, Height, Scene, Depth)
%% (raytracer.erl:86-178, chosen by tracing_function/1 at :714-719, called by raytrace/5
%% at :723-733).  raytracer.erl itself is not edited:
%%
%%   raytracer:raytrace(640, 480, "/tmp/traced.ppm", 3, fun raytracer_gpu:raytraced_pixel_list_gpu/4).
%%   raytracer_gpu:go(640, 480, "/tmp/traced.ppm", 3).
%%
%% The returned list is exactly what the reference strategies return: the concurrent and
%% distributed forms key each pixel by X+Y*Width and sort by key (raytracer.erl:112, :155,
%% :173), the simple form uses key 1 (raytracer.erl:95); write_pixels_to_ppm/5 ignores keys.
-module(raytracer_gpu).
-export([raytraced_pixel_list_gpu/4,
         raytraced_pixel_list_simple/4,
         raytraced_pixel_list_concurrent/4,
         raytraced_pixel_list_distributed/4,
         render_binary/4,
         go/4]).
-on_load(init/0).

init() ->
    Priv = case code:priv_dir(raytracer_gpu) of
               {error, _} -> filename:join(filename:dirname(filename:dirname(code:which(?MODULE))), "priv");
               Dir -> Dir
           end,
    erlang:load_nif(filename:join(Priv, "rt_nif"), 0).

%% the new strategy: one GPU render, pixels keyed X+Y*Width in row-major order
raytraced_pixel_list_gpu(Width, Height, Scene, Recursion_depth) ->
    rt_nif:render(Width, Height, Scene, Recursion_depth, indexed).

raytraced_pixel_list_simple(Width, Height, Scene, Recursion_depth) ->
    rt_nif:render(Width, Height, Scene, Recursion_depth, simple).

raytraced_pixel_list_concurrent(Width, Height, Scene, Recursion_depth) ->
    rt_nif:render(Width, Height, Scene, Recursion_depth, indexed).

%% rows are shared over every GPU the library sees (rt_opts.ndev = -1)
raytraced_pixel_list_distributed(Width, Height, Scene, Recursion_depth) ->
    rt_nif:render(Width, Height, Scene, Recursion_depth, distributed).

%% W*H*3 native-endian doubles, row-major: for frames too large for a tuple list
render_binary(Width, Height, Scene, Recursion_depth) ->
    rt_nif:render_binary(Width, Height, Scene, Recursion_depth).

go(Width, Height, Filename, Recursion_depth) ->
    raytracer:raytrace(Width, Height, Filename, Recursion_depth, fun raytraced_pixel_list_gpu/4).
