%% psim_philox -- the simulator's RNG as an OTP `rand` algorithm, so the
%% reference modules draw exactly the values the engine and the oracle draw.
%%
%% A node's manager stream is Philox4x32-10 with key = the 64-bit seed and
%% counter = (draw# low, draw# high, node id, 0); a draw is the top 58 bits
%% of the first two output words (exsplus width, partisan_config.erl:154-170
%% seeds exsplus).  rand:uniform/0,1 are OTP's own mappings over `bits` = 58
%% (rand.erl ?uniform_range; float = V bsr 5 * 2^-53), the same as
%% partisan_amd/csrc/psim_device.h draw58_at and oracle/psim_oracle.c.
-module(psim_philox).
-export([install/3, state/0, philox/6, draw58/3]).

-define(M32, 16#FFFFFFFF).

%% install the stream of Node at draw counter Ctr into this process's
%% rand state (the process dictionary key rand_seed, as rand:seed/1 does)
install(Seed, Node, Ctr) ->
    Alg = #{type => psim_philox, bits => 58, next => fun next/1},
    put(rand_seed, {Alg, {Seed, Node, Ctr}}),
    ok.

%% {Seed, Node, Ctr} of the installed stream (the draw counter to save)
state() ->
    {_, S} = get(rand_seed),
    S.

next({Seed, Node, Ctr}) ->
    {draw58(Seed, Node, Ctr), {Seed, Node, Ctr + 1}}.

draw58(Seed, Node, Ctr) ->
    {O0, O1} = philox(Ctr band ?M32, (Ctr bsr 32) band ?M32, Node, 0, Seed band ?M32, (Seed bsr 32) band ?M32),
    ((O1 bsl 32) bor O0) bsr 6.

%% Philox4x32-10, the first two output words (Random123 KATs:
%% tests/golden/philox4x32_10_kat.json)
philox(C0, C1, C2, C3, K0, K1) -> rounds(10, C0, C1, C2, C3, K0, K1).

rounds(0, C0, C1, _C2, _C3, _K0, _K1) -> {C0, C1};
rounds(N, C0, C1, C2, C3, K0, K1) ->
    P0 = 16#D2511F53 * C0,
    P1 = 16#CD9E8D57 * C2,
    N0 = ((P1 bsr 32) bxor C1 bxor K0) band ?M32,
    N2 = ((P0 bsr 32) bxor C3 bxor K1) band ?M32,
    rounds(N - 1, N0, P1 band ?M32, N2, P0 band ?M32,
           (K0 + 16#9E3779B9) band ?M32, (K1 + 16#BB67AE85) band ?M32).
