%% partisan_gpu_sim -- NIF bindings of the MI355X simulator
%% (include/partisan_gpu_sim.h).  Node ids are the simulated nodes; an id maps
%% to the harness node_spec #{name => 'n<id>@sim', ...} (DESIGN.md section 2).
-module(partisan_gpu_sim).
-export([create/1, join/3, crash/2, revive/2, leave/2, leave_node/3, broadcast/3, step/2, active/2, members/3,
         delivery/2, histograms/1, snapshot/1, restore/2, set_partition/2, clear_partition/1, node/2,
         begin_send_omission/3, end_send_omission/3, begin_receive_omission/3, end_receive_omission/3,
         begin_omission/2, end_omission/2, clear_faults/1]).
-on_load(init/0).

init() ->
    Priv = case code:priv_dir(partisan_gpu_sim) of
               {error, _} -> "priv";
               Dir -> Dir
           end,
    erlang:load_nif(filename:join(Priv, "partisan_gpu_sim_nif"), 0).

-spec create(map()) -> {ok, reference()} | {error, atom()}.
create(_Config) -> erlang:nif_error(nif_not_loaded).

%% Nodes/Contacts: lists of ids, packed as little-endian u32 binaries.
join(Sim, Nodes, Contacts) -> join_nif(Sim, pack(Nodes), pack(Contacts)).
crash(Sim, Nodes) -> crash_nif(Sim, pack(Nodes)).
%% restart without a join (init/1 state; reached through passive views)
revive(Sim, Nodes) -> revive_nif(Sim, pack(Nodes)).
%% leave/0 at each node (pluggable manager handles; {error, unsupported} on HyParView)
leave(Sim, Nodes) -> leave_nif(Sim, pack(Nodes)).
%% leave/1 at each actor: Actors[i] removes Targets[i] (SCAMP v1 / v2 handles)
leave_node(Sim, Actors, Targets) -> leave_node_nif(Sim, pack(Actors), pack(Targets)).
broadcast(_Sim, _Root, _Id) -> erlang:nif_error(nif_not_loaded).
step(_Sim, _Rounds) -> erlang:nif_error(nif_not_loaded).
active(_Sim, _Node) -> erlang:nif_error(nif_not_loaded).
%% pluggable manager handles: the strategy membership of Node (N = n_nodes)
members(_Sim, _Node, _N) -> erlang:nif_error(nif_not_loaded).
%% the tracked broadcast at Node: {ok, {Have, FirstRound, Hop}}
delivery(_Sim, _Node) -> erlang:nif_error(nif_not_loaded).
%% overlay statistics (psim_histograms) as a map
histograms(_Sim) -> erlang:nif_error(nif_not_loaded).
%% whole-simulation state as a binary, and back into a handle of the same config
snapshot(_Sim) -> erlang:nif_error(nif_not_loaded).
restore(_Sim, _Bin) -> erlang:nif_error(nif_not_loaded).

%% the partition group of every node (a list of N small integers): an
%% injected partition as a network partition (DESIGN.md section 2);
%% clear_partition/1 resolves it
set_partition(Sim, Groups) -> set_partition_nif(Sim, << <<G:8>> || G <- Groups >>).
clear_partition(_Sim) -> erlang:nif_error(nif_not_loaded).
%% one node: {ok, #{up, epoch, active, passive, have, round}}
node(_Sim, _Node) -> erlang:nif_error(nif_not_loaded).

%% omission faults of the pluggable manager's interposition layer (the
%% crash-fault model's commands, test/prop_partisan_crash_fault_model.erl
%% :93-229), pairwise over lists of ids; pluggable handles only
begin_send_omission(Sim, Srcs, Dsts) -> omission_nif(Sim, 0, pack(Srcs), pack(Dsts), 1).
end_send_omission(Sim, Srcs, Dsts) -> omission_nif(Sim, 0, pack(Srcs), pack(Dsts), 0).
begin_receive_omission(Sim, Srcs, Dsts) -> omission_nif(Sim, 1, pack(Srcs), pack(Dsts), 1).
end_receive_omission(Sim, Srcs, Dsts) -> omission_nif(Sim, 1, pack(Srcs), pack(Dsts), 0).
begin_omission(Sim, Nodes) -> faulted_nif(Sim, pack(Nodes), 1).
end_omission(Sim, Nodes) -> faulted_nif(Sim, pack(Nodes), 0).
%% resolve_all_faults_with_heal
clear_faults(_Sim) -> erlang:nif_error(nif_not_loaded).

pack(Ids) -> << <<I:32/little>> || I <- Ids >>.
omission_nif(_S, _K, _A, _B, _On) -> erlang:nif_error(nif_not_loaded).
faulted_nif(_S, _N, _On) -> erlang:nif_error(nif_not_loaded).
set_partition_nif(_S, _G) -> erlang:nif_error(nif_not_loaded).
join_nif(_S, _N, _C) -> erlang:nif_error(nif_not_loaded).
crash_nif(_S, _N) -> erlang:nif_error(nif_not_loaded).
revive_nif(_S, _N) -> erlang:nif_error(nif_not_loaded).
leave_nif(_S, _N) -> erlang:nif_error(nif_not_loaded).
leave_node_nif(_S, _A, _T) -> erlang:nif_error(nif_not_loaded).
