%% rt_nif.erl — Erlang side of the NIF in erlang/c_src/rt_nif.c (the only module that loads it:
%% ERL_NIF_INIT(rt_nif, ...) names this module).
-module(rt_nif).
-export([render_frame/5, pixels_chunk/5, render_binary/4, render_binary/5, render_ppm_file/5]).
-on_load(init/0).

init() ->
    Priv = case code:priv_dir(raytracer_gpu) of
               {error, _} -> filename:join(filename:dirname(filename:dirname(code:which(?MODULE))), "priv");
               Dir -> Dir
           end,
    erlang:load_nif(filename:join(Priv, "rt_nif"), 0).

%% render_frame(Width, Height, Scene, Depth, #{spp => N, seed => S, devices => all | N})
%%   -> done | {rt_frame, Width, Height, Rgb, Levels, Lights}
%% Rgb: W*H*3 native-endian doubles, row-major (pinned host memory); Levels: one byte per pixel.
render_frame(_Width, _Height, _Scene, _Depth, _Opts) ->
    erlang:nif_error(nif_not_loaded).

%% pixels_chunk(Frame, Start, Count, simple | indexed, Tail) -> [{Key, {R, G, B}} | Tail]
pixels_chunk(_Frame, _Start, _Count, _KeyMode, _Tail) ->
    erlang:nif_error(nif_not_loaded).

%% render_binary(Width, Height, Scene, Depth) -> done | binary()
render_binary(_Width, _Height, _Scene, _Depth) ->
    erlang:nif_error(nif_not_loaded).

%% render_binary(Width, Height, Scene, Depth, #{spp => N, seed => S, devices => all | N}) -> done | binary()
%% Stochastic supersampling as defined at RT_SUPERSAMPLING in include/rt_mi355x.h.
render_binary(_Width, _Height, _Scene, _Depth, _Opts) ->
    erlang:nif_error(nif_not_loaded).

%% render_ppm_file(Width, Height, Scene, Depth, Filename) -> ok | done
%% raytrace/5's render plus write_pixels_to_ppm/5 (MaxValue 255), the P3 text made on the GPU.
render_ppm_file(_Width, _Height, _Scene, _Depth, _Filename) ->
    erlang:nif_error(nif_not_loaded).
