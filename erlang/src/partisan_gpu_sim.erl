%% partisan_gpu_sim -- NIF bindings of the MI355X simulator
%% (include/partisan_gpu_sim.h).  Node ids are the simulated nodes; an id maps
%% to the harness node_spec #{name => 'n<id>@sim', ...} (DESIGN.md section 2).
%%
%% The short NIFs run on normal schedulers and answer {error, busy} while
%% another process holds the handle inside a step (dirty scheduler).  Every
%% wrapper below goes through call/1, which retries a busy answer with a
%% bounded back-off, so callers may match on success directly.
-module(partisan_gpu_sim).
-export([create/1, join/3, crash/2, revive/2, leave/2, leave_node/3, broadcast/3, step/2, active/2, members/3,
         delivery/2, histograms/1, snapshot/1, restore/2, set_partition/2, clear_partition/1, node/2,
         begin_send_omission/3, end_send_omission/3, begin_receive_omission/3, end_receive_omission/3,
         begin_omission/2, end_omission/2, clear_faults/1, msg_slots/1, set_bucket_table/2, phash_buckets/2,
         set_phash_table/2, phash_table/2, spec_ip/1]).
-on_load(init/0).

%% back-off of a busy handle: 1 ms sleeps, at most ~10 s in all
-define(BUSY_TRIES, 10000).

init() ->
    Priv = case code:priv_dir(partisan_gpu_sim) of
               {error, _} -> "priv";
               Dir -> Dir
           end,
    erlang:load_nif(filename:join(Priv, "partisan_gpu_sim_nif"), 0).

-spec create(map()) -> {ok, reference()} | {error, atom()}.
create(_Config) -> erlang:nif_error(nif_not_loaded).

%% Nodes/Contacts: lists of ids, packed as little-endian u32 binaries.
join(Sim, Nodes, Contacts) -> call(fun() -> join_nif(Sim, pack(Nodes), pack(Contacts)) end).
crash(Sim, Nodes) -> call(fun() -> crash_nif(Sim, pack(Nodes)) end).
%% restart without a join (init/1 state; reached through passive views)
revive(Sim, Nodes) -> call(fun() -> revive_nif(Sim, pack(Nodes)) end).
%% leave/0 at each node (pluggable manager handles; {error, unsupported} on HyParView)
leave(Sim, Nodes) -> call(fun() -> leave_nif(Sim, pack(Nodes)) end).
%% leave/1 at each actor: Actors[i] removes Targets[i] (SCAMP v1 / v2 handles)
leave_node(Sim, Actors, Targets) -> call(fun() -> leave_node_nif(Sim, pack(Actors), pack(Targets)) end).
broadcast(Sim, Root, Id) -> call(fun() -> broadcast_nif(Sim, Root, Id) end).
%% a dirty NIF: waits for the handle's mutex itself
step(_Sim, _Rounds) -> erlang:nif_error(nif_not_loaded).
active(Sim, Node) -> call(fun() -> active_nif(Sim, Node) end).
%% pluggable manager handles: the strategy membership of Node (N = n_nodes)
members(Sim, Node, N) -> call(fun() -> members_nif(Sim, Node, N) end).
%% the tracked broadcast at Node: {ok, {Have, FirstRound, Hop}}
delivery(Sim, Node) -> call(fun() -> delivery_nif(Sim, Node) end).
%% overlay statistics (psim_histograms) as a map (dirty NIF)
histograms(_Sim) -> erlang:nif_error(nif_not_loaded).
%% whole-simulation state as a binary, and back into a handle of the same config (dirty NIFs)
snapshot(_Sim) -> erlang:nif_error(nif_not_loaded).
restore(_Sim, _Bin) -> erlang:nif_error(nif_not_loaded).

%% the partition group of every node (a list of N small integers): an
%% injected partition as a network partition (DESIGN.md section 2);
%% clear_partition/1 resolves it
set_partition(Sim, Groups) ->
    Bin = << <<G:8>> || G <- Groups >>,
    call(fun() -> set_partition_nif(Sim, Bin) end).
clear_partition(Sim) -> call(fun() -> clear_partition_nif(Sim) end).
%% the sets v1 order of every view (SURVEY App. A Q1): one bucket per node,
%% erlang:phash(NodeSpec, 16) - 1, before the first step
set_bucket_table(Sim, Buckets) ->
    Bin = << <<B:8>> || B <- Buckets >>,
    call(fun() -> set_bucket_table_nif(Sim, Bin) end).
%% that table for node specs Spec(0) .. Spec(N - 1), computed by this VM
phash_buckets(N, Spec) -> [erlang:phash(Spec(I), 16) - 1 || I <- lists:seq(0, N - 1)].
%% the whole hash, erlang:phash(NodeSpec, 2^32) - 1 per node: the slots of
%% every sets v1 set the engine keeps, SCAMP v1 memberships past 80 ids
%% included (OTP's linear hash, psim_set_phash_table); before the first step
set_phash_table(Sim, Hashes) ->
    Bin = << <<H:32/native>> || H <- Hashes >>,
    call(fun() -> set_phash_table_nif(Sim, Bin) end).
phash_table(N, Spec) -> [erlang:phash(Spec(I), 4294967296) - 1 || I <- lists:seq(0, N - 1)].
%% the simulated node_spec's listen address: 10.0.0.0 + Id, so that term
%% order (the ip tuple decides it: listen_addrs precedes name) is id order for
%% every id below 2^27 (psim_wire.cpp's ip_base + id)
spec_ip(Id) ->
    Ip = 16#0A000000 + Id,
    {Ip bsr 24, (Ip bsr 16) band 255, (Ip bsr 8) band 255, Ip band 255}.
%% one node: {ok, #{up, epoch, active, passive, have, round}}
node(Sim, Node) -> call(fun() -> node_nif(Sim, Node) end).
%% the live message slots: {ok, [{Slot, MsgId, RootId}]} -- delivery bit
%% Slot of node/2's `have` answers for MsgId only (psim_get_msg_slots)
msg_slots(Sim) -> call(fun() -> msg_slots_nif(Sim) end).

%% omission faults of the pluggable manager's interposition layer (the
%% crash-fault model's commands, test/prop_partisan_crash_fault_model.erl
%% :93-229), pairwise over lists of ids; pluggable handles only
begin_send_omission(Sim, Srcs, Dsts) -> omission(Sim, 0, Srcs, Dsts, 1).
end_send_omission(Sim, Srcs, Dsts) -> omission(Sim, 0, Srcs, Dsts, 0).
begin_receive_omission(Sim, Srcs, Dsts) -> omission(Sim, 1, Srcs, Dsts, 1).
end_receive_omission(Sim, Srcs, Dsts) -> omission(Sim, 1, Srcs, Dsts, 0).
begin_omission(Sim, Nodes) -> call(fun() -> faulted_nif(Sim, pack(Nodes), 1) end).
end_omission(Sim, Nodes) -> call(fun() -> faulted_nif(Sim, pack(Nodes), 0) end).
%% resolve_all_faults_with_heal
clear_faults(Sim) -> call(fun() -> clear_faults_nif(Sim) end).

omission(Sim, Kind, Srcs, Dsts, On) ->
    S = pack(Srcs),
    D = pack(Dsts),
    call(fun() -> omission_nif(Sim, Kind, S, D, On) end).

%% a short NIF, retried while the handle is inside another process's step
call(F) -> call(F, ?BUSY_TRIES).

call(F, Tries) ->
    case F() of
        {error, busy} when Tries > 1 ->
            timer:sleep(1),
            call(F, Tries - 1);
        Result ->
            Result
    end.

pack(Ids) -> << <<I:32/little>> || I <- Ids >>.
omission_nif(_S, _K, _A, _B, _On) -> erlang:nif_error(nif_not_loaded).
faulted_nif(_S, _N, _On) -> erlang:nif_error(nif_not_loaded).
set_partition_nif(_S, _G) -> erlang:nif_error(nif_not_loaded).
join_nif(_S, _N, _C) -> erlang:nif_error(nif_not_loaded).
crash_nif(_S, _N) -> erlang:nif_error(nif_not_loaded).
revive_nif(_S, _N) -> erlang:nif_error(nif_not_loaded).
leave_nif(_S, _N) -> erlang:nif_error(nif_not_loaded).
leave_node_nif(_S, _A, _T) -> erlang:nif_error(nif_not_loaded).
broadcast_nif(_S, _R, _I) -> erlang:nif_error(nif_not_loaded).
active_nif(_S, _N) -> erlang:nif_error(nif_not_loaded).
members_nif(_S, _N, _K) -> erlang:nif_error(nif_not_loaded).
delivery_nif(_S, _N) -> erlang:nif_error(nif_not_loaded).
clear_partition_nif(_S) -> erlang:nif_error(nif_not_loaded).
set_bucket_table_nif(_S, _B) -> erlang:nif_error(nif_not_loaded).
set_phash_table_nif(_S, _B) -> erlang:nif_error(nif_not_loaded).
clear_faults_nif(_S) -> erlang:nif_error(nif_not_loaded).
node_nif(_S, _N) -> erlang:nif_error(nif_not_loaded).
msg_slots_nif(_S) -> erlang:nif_error(nif_not_loaded).
