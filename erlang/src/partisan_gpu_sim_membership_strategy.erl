%% partisan_gpu_sim_membership_strategy -- the partisan_membership_strategy
%% behaviour (src/partisan_membership_strategy.erl:32-36) backed by the MI355X
%% simulator.  One simulator handle (manager = pluggable, strategy = full /
%% scamp v1 / scamp v2 from partisan_config) holds every simulated node; this
%% module answers the callbacks of one of them (`sim_node`), so the pluggable
%% manager (pluggable:384, :886, :1001, :1162, :1398) can be pointed at it
%% with partisan_config:set(membership_strategy, ?MODULE).
%%
%% The simulator runs the strategy's own message exchange on the GPU, so the
%% outgoing-message lists returned here are empty: the manager has nothing to
%% forward.  periodic/1 advances the whole overlay by one round (R0-P,
%% DESIGN.md section 2b) -- call it from one node only (the `sim_driver`).
-module(partisan_gpu_sim_membership_strategy).
-behaviour(partisan_membership_strategy).

-export([init/1, join/3, leave/2, periodic/1, handle_message/2]).
-export([start_seed/1]).

-record(sim_strategy, {sim, me :: non_neg_integer(), n :: pos_integer(), driver :: boolean(),
                       started = false :: boolean()}).

-define(NONE, 16#FFFFFFFF).

%% The node starts in the simulator exactly once: at join/3 with its contact,
%% or -- a seed that never joins -- at init/1 when partisan_config's
%% `sim_seed_node` is true (or later through start_seed/1).  Until then it is
%% inert: periodic/1 and handle_message/2 answer [Myself] and start nothing,
%% so a periodic tick that comes before the user's join (the pluggable
%% manager schedules periodic from init, pl:363) cannot turn a joiner into a
%% singleton.  join/3 on a node already started (a seed, or a second join)
%% cannot be expressed in the simulator -- psim_join would restart the node,
%% and a full-strategy node cannot restart at all -- so it raises
%% {already_started, Me} instead of reporting a join that did not happen.
init(_Identity) ->
    N = partisan_config:get(sim_nodes, 32),
    Me = partisan_config:get(sim_node, 0),
    Strategy = case partisan_config:get(membership_strategy_sim, full) of
                   full -> 0; scamp_v1 -> 1; scamp_v2 -> 2
               end,
    {ok, Sim} = case partisan_config:get(sim_handle, undefined) of
                    undefined ->
                        {ok, H0} = partisan_gpu_sim:create(#{n_nodes => N, seed => partisan_config:get(sim_seed, 1),
                                                             manager => 1, strategy => Strategy,
                                                             fanout => partisan_config:get(sim_fanout, 0),
                                                             scamp_c => partisan_config:get(scamp_c, 5),
                                                             periodic_interval => 10}),
                        %% SCAMP v1's membership in this VM's sets v1 order
                        %% (SURVEY App. A Q1; OTP's linear hash past 80 ids)
                        ok = partisan_gpu_sim:set_phash_table(H0, partisan_gpu_sim:phash_table(N, fun spec/1)),
                        {ok, H0};
                    H -> {ok, H}
                end,
    State0 = #sim_strategy{sim = Sim, me = Me, n = N,
                           driver = partisan_config:get(sim_driver, false)},
    State = case partisan_config:get(sim_seed_node, false) of
                true -> start_seed(State0);
                false -> State0
            end,
    {ok, membership(State), State}.

%% a seed: the node starts alone (no contact) in the next round
start_seed(State = #sim_strategy{started = false, sim = Sim, me = Me}) ->
    ok = partisan_gpu_sim:join(Sim, [Me], [?NONE]),
    State#sim_strategy{started = true};
start_seed(State) ->
    State.

%% Strategy:join/3 at the joiner: the simulated hello/state handshake and the
%% strategy's join happen in the next rounds of the simulator.  A join of a
%% node already started is refused loudly (see the header).
join(#sim_strategy{started = true, me = Me}, _Node, _RemoteState) ->
    erlang:error({already_started, Me});
join(State = #sim_strategy{sim = Sim, me = Me}, #{name := Name}, _RemoteState) ->
    ok = partisan_gpu_sim:join(Sim, [Me], [id(Name)]),
    State1 = State#sim_strategy{started = true},
    {ok, membership(State1), [], State1}.

%% leave/2: the pluggable manager calls it from handle_call({leave, Node})
%% (pluggable:502-515).  Node = myself is leave/0 (the node stops in the next
%% round, psim_leave); another node is leave/1 at this node (psim_leave_node).
leave(State = #sim_strategy{sim = Sim, me = Me}, #{name := Name}) ->
    ok = case id(Name) of
             Me -> partisan_gpu_sim:leave(Sim, [Me]);
             T -> partisan_gpu_sim:leave_node(Sim, [Me], [T])
         end,
    {ok, membership(State), [], State}.

periodic(State = #sim_strategy{sim = Sim, driver = true}) ->
    {ok, _Stats} = partisan_gpu_sim:step(Sim, 1),
    {ok, membership(State), [], State};
periodic(State) ->
    {ok, membership(State), [], State}.

%% messages between simulated nodes never leave the GPU
handle_message(State, _Message) ->
    {ok, membership(State), [], State}.

membership(#sim_strategy{started = false, me = Me}) ->
    [spec(Me)];                                              % init/1: [Myself]
membership(#sim_strategy{sim = Sim, me = Me, n = N}) ->
    {ok, Ids} = partisan_gpu_sim:members(Sim, Me, N),
    [spec(I) || I <- Ids].

spec(I) ->
    #{name => name(I), listen_addrs => [#{ip => partisan_gpu_sim:spec_ip(I), port => 9090}],
       channels => [undefined], parallelism => 1}.

name(Id) -> list_to_atom(lists:flatten(io_lib:format("n~10..0B@sim", [Id]))).
id(Name) ->
    [$n | Rest] = atom_to_list(Name),
    list_to_integer(lists:takewhile(fun(C) -> C >= $0 andalso C =< $9 end, Rest)).
