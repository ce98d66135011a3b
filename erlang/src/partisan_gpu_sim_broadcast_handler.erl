%% partisan_gpu_sim_broadcast_handler -- the partisan_plumtree_broadcast_handler
%% behaviour (src/partisan_plumtree_broadcast_handler.erl:23-43) for broadcasts
%% simulated on the MI355X.  Plumtree itself (eager/lazy push, PRUNE, IHAVE,
%% GRAFT: src/partisan_plumtree_broadcast.erl) runs on the GPU for every
%% simulated node; this module answers the handler callbacks for one of them
%% (`sim_node`), with the delivery state the simulator keeps in place of
%% partisan_plumtree_backend's ETS table (plumtree_backend:101-108, :140-167).
%%
%% Messages follow the backend's heartbeat shape: the id is
%% {RootName, Counter} (plumtree_backend:179-200) and the payload is the id.
%% Counter is the simulator's 16-bit message id; the delivery state of a node
%% is a mask over Counter mod 64 (PSIM_MSG_SLOTS, DESIGN.md section 2).
%%
%%   broadcast_data/1  {Id, Payload} of a #sim_broadcast{}        (handler :23-24)
%%   merge/2           true iff the simulated node had not yet
%%                     received Id (the device merged it on delivery:
%%                     the handler reports, it cannot deliver)  (handler :26-28)
%%   is_stale/1        Id already received                      (handler :30-32)
%%   graft/1           {ok, Payload} when received, else {error, {not_found, Id}}
%%                     -- as plumtree_backend:148-157 (no `stale` answer)
%%   exchange/1        the backend's no-op exchange: a process that exits
%%                     at once (plumtree_backend:112-124)
%%
%% broadcast/1 originates a broadcast at the simulated node (the backend's
%% heartbeat, plumtree_backend:179-200): psim_broadcast in the next round.
-module(partisan_gpu_sim_broadcast_handler).
-behaviour(partisan_plumtree_broadcast_handler).

-export([broadcast_data/1, merge/2, is_stale/1, graft/1, exchange/1]).
-export([broadcast/1, sim_broadcast/1]).

-record(sim_broadcast, {root :: atom(), counter :: non_neg_integer()}).

broadcast_data(#sim_broadcast{root = Root, counter = C}) ->
    Id = {Root, C},
    {Id, Id}.

merge(Id, _Payload) ->
    not is_stale(Id).

%% Counter's slot must still hold Counter: a retired id (its slot taken by
%% a newer broadcast, Counter - 64k) is one the backend no longer knows --
%% stale for is_stale/1 (the engine treats it so, counting an overflow) and
%% not graftable
is_stale({_Root, Counter}) ->
    case delivered(Counter) of
        retired -> true;
        Have -> Have
    end.

graft(Id = {_Root, Counter}) ->
    case delivered(Counter) of
        true -> {ok, Id};
        _ -> {error, {not_found, Id}}
    end.

%% true / false: the simulated node's delivery bit of a live id; retired
delivered(Counter) ->
    {Sim, Me} = handle(),
    Slot = Counter rem 64,
    {ok, Slots} = partisan_gpu_sim:msg_slots(Sim),
    case lists:keyfind(Slot, 1, Slots) of
        {Slot, Counter, _Root} ->
            {ok, #{have := Have}} = partisan_gpu_sim:node(Sim, Me),
            (Have bsr Slot) band 1 =:= 1;
        _ ->
            retired
    end.

exchange(_Peer) ->
    Pid = spawn_link(fun() -> ok end),
    {ok, Pid}.

%% originate broadcast Counter at the simulated node (Counter < 65536)
broadcast(Counter) when is_integer(Counter), Counter >= 0, Counter < 65536 ->
    {Sim, Me} = handle(),
    case partisan_gpu_sim:broadcast(Sim, Me, Counter) of
        ok -> {ok, sim_broadcast(Counter)};
        Error -> Error
    end.

sim_broadcast(Counter) ->
    #sim_broadcast{root = partisan_peer_service_manager:mynode(), counter = Counter}.

handle() ->
    {ok, Sim} = partisan_gpu_sim_peer_service_manager:sim(),
    {Sim, partisan_config:get(sim_node, 0)}.
