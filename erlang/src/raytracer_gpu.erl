%% raytracer_gpu.erl — the MI355X strategy funs for the reference ray tracer
%% (plouj/eraytracer, raytracer.erl), backed by the rt_nif NIF (erlang/c_src/rt_nif.c)
%% and the HIP library librtmi355x.so.  This module does not load the NIF itself:
%% rt_nif (whose ERL_NIF_INIT names it) does, on its own load.
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
%% Term types are the reference's too: {0,0,0} integers for background, depth-0 and no-light
%% pixels, floats elsewhere (rt_nif.c); a supersampled frame (Opts spp > 1, which the reference
%% does not have) is floats everywhere.
%%
%% Result delivery (the reference's master sends one W*H list, :116-118, :155): the frame
%% comes back once as a binary (render_frame/5); the list is then built from the end in
%% chunks of ?CHUNK pixels, each a short NIF call (no multi-million-tuple build inside one
%% call), or consumed without building it: fold_pixels/4 folds chunk by chunk, and
%% pixel_stream/2 is a lazy list of chunks.
-module(raytracer_gpu).
-export([raytraced_pixel_list_gpu/4,
         raytraced_pixel_list_simple/4,
         raytraced_pixel_list_concurrent/4,
         raytraced_pixel_list_distributed/4,
         render_frame/4, render_frame/5,
         pixel_list/2, fold_pixels/4, pixel_stream/2,
         render_binary/4,
         go/4]).

-define(CHUNK, 4096). % <= rt_nif.c PIXELS_CHUNK_MAX: one chunk stays within a NIF timeslice

%% the new strategy: one GPU render, pixels keyed X+Y*Width in row-major order
raytraced_pixel_list_gpu(Width, Height, Scene, Recursion_depth) ->
    strategy(Width, Height, Scene, Recursion_depth, indexed, #{}).

raytraced_pixel_list_simple(Width, Height, Scene, Recursion_depth) ->
    strategy(Width, Height, Scene, Recursion_depth, simple, #{}).

raytraced_pixel_list_concurrent(Width, Height, Scene, Recursion_depth) ->
    strategy(Width, Height, Scene, Recursion_depth, indexed, #{}).

%% rows are shared over every GPU the library sees (rt_opts.ndev = -1)
raytraced_pixel_list_distributed(Width, Height, Scene, Recursion_depth) ->
    strategy(Width, Height, Scene, Recursion_depth, indexed, #{devices => all}).

strategy(Width, Height, Scene, Recursion_depth, KeyMode, Opts) ->
    case render_frame(Width, Height, Scene, Recursion_depth, Opts) of
        done -> done;
        Frame -> pixel_list(Frame, KeyMode)
    end.

render_frame(Width, Height, Scene, Recursion_depth) ->
    render_frame(Width, Height, Scene, Recursion_depth, #{}).

render_frame(Width, Height, Scene, Recursion_depth, Opts) ->
    rt_nif:render_frame(Width, Height, Scene, Recursion_depth, Opts).

%% The whole [{Key, {R,G,B}}] list, built from the last chunk to the first (each chunk is
%% consed onto the list built so far, so nothing is appended or copied).
pixel_list({rt_frame, W, H, _, _, _} = Frame, KeyMode) ->
    build(Frame, KeyMode, W * H, []).

build(_Frame, _KeyMode, 0, Acc) ->
    Acc;
build(Frame, KeyMode, End, Acc) ->
    Start = max(0, End - ?CHUNK),
    build(Frame, KeyMode, Start, rt_nif:pixels_chunk(Frame, Start, End - Start, KeyMode, Acc)).

%% Fun({Key, {R,G,B}}, Acc) over the pixels in row-major order, one chunk built at a time.
fold_pixels(Fun, Acc0, {rt_frame, W, H, _, _, _} = Frame, KeyMode) ->
    fold_chunks(Fun, Acc0, Frame, KeyMode, 0, W * H).

fold_chunks(_Fun, Acc, _Frame, _KeyMode, N, N) ->
    Acc;
fold_chunks(Fun, Acc, Frame, KeyMode, Start, N) ->
    Count = min(?CHUNK, N - Start),
    Acc1 = lists:foldl(Fun, Acc, rt_nif:pixels_chunk(Frame, Start, Count, KeyMode, [])),
    fold_chunks(Fun, Acc1, Frame, KeyMode, Start + Count, N).

%% A lazy list of chunks: [] at the end, otherwise {Chunk, Next} with Next() the rest.
pixel_stream({rt_frame, W, H, _, _, _} = Frame, KeyMode) ->
    stream(Frame, KeyMode, 0, W * H).

stream(_Frame, _KeyMode, N, N) ->
    [];
stream(Frame, KeyMode, Start, N) ->
    Count = min(?CHUNK, N - Start),
    {rt_nif:pixels_chunk(Frame, Start, Count, KeyMode, []),
     fun() -> stream(Frame, KeyMode, Start + Count, N) end}.

%% W*H*3 native-endian doubles, row-major: for frames too large for a tuple list
render_binary(Width, Height, Scene, Recursion_depth) ->
    rt_nif:render_binary(Width, Height, Scene, Recursion_depth).

go(Width, Height, Filename, Recursion_depth) ->
    raytracer:raytrace(Width, Height, Filename, Recursion_depth, fun raytraced_pixel_list_gpu/4).
