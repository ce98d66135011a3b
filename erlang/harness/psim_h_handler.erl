%% The Plumtree handler module of the parity harness: partisan_plumtree_backend
%% semantics (plumtree_backend:81-124, :140-167) with one received-id set per
%% simulated node instead of one ETS table per VM.
-module(psim_h_handler).
-behaviour(partisan_plumtree_broadcast_handler).
-export([broadcast_data/1, merge/2, is_stale/1, graft/1, exchange/1]).

broadcast_data({psim_msg, Id}) -> {Id, Id}.

merge(Id, Id) ->
    case is_stale(Id) of
        true -> false;
        false -> psim_harness:have_add(Id), true
    end.

is_stale(Id) -> psim_harness:have(Id).

graft(Id) ->
    case is_stale(Id) of
        true -> {ok, Id};
        false -> {error, {not_found, Id}}
    end.

exchange(_Peer) -> {ok, spawn_link(fun() -> ok end)}.
